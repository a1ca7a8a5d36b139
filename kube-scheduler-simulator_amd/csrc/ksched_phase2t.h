// Phase 2, transposed walk (KSG_BATCH_MODE=tcol; the default for runs whose
// ranges pass the N32 check), included by ksched.hip inside its anonymous
// namespace after ksg_batch_phase2s.
//
// The slot walk (ksg_batch_phase2s) gives each changed node a lane and, per
// pod, re-evaluates the pod on every changed node, reduces across the lanes and
// workgroup, and decides: a full evaluation, a block reduction and a barrier
// sit on the per-pod chain.  Here the roles are swapped: ONE wave, lane l
// holds the batch's pods l and l + 64 (P = 2), and a changed node is a column.
// Pod k's decision needs, besides the best unchanged node of its top set T_k
// (phase 1 + top-k, as in the slot walk), the best of its columns: the nodes
// D chosen by pods 0..k-1, evaluated for pod k on their live rows.  Every
// column value is computed ONCE, when its node is assumed onto: right after
// pod k's assume, every lane evaluates its pods q > k on that node's new row
// (the same exact 32-bit Fit / BalancedAllocation as the slot walk's N32
// instances), and folds the value into a per-pod running top-2 over the
// columns.  The per-pod chain is then: read lane k's best column (v_readlane),
// compare with the best unchanged key, assume, evaluate one column, update the
// running maxima.  No cross-lane reduction and no barrier is on it.
//
//   * Per-pod running maxima: B1 (best live column key, with its slot), B2
//     (the best over the other columns, exact while `x2`).  A node assumed onto
//     again (a re-choice) rewrites its column; the cases that leave B1 unknown
//     (the holder re-chosen and its value fell, with B2 inexact) set a rescan
//     flag, and the pod's maxima are recomputed from the stored columns before
//     its decision (rare).
//   * Column store (LDS, [slot][pod] u32): phase-1 static total part `stat`
//     (14 bits), live total (14 bits), phase-1 feasible, live feasible, and
//     whether the node held the pod's phase-1 TaintToleration / NodeAffinity
//     maximum: a re-choice needs no global load, and the per-pod counters
//     (feasible at phase 1, live, lost maximum holders) are exact, as in the
//     slot walk.
//   * Loads: after pod k's assume the best unchanged node of pod k + 1 is
//     known exactly (T_{k+1}'s first entry outside D); its phase-1 records for
//     every pod and its columns are fetched then, a full step before the
//     column evaluation that needs them if pod k + 1 takes it.  A re-choice
//     reads the column store; anything else (the rare paths) loads on demand.
//   * The renormalisation case (a phase-1 maximum whose every holder became
//     infeasible, or a range error) rescans pod k's phase-1 records with the
//     live maxima, as the slot walk does; the live part of a changed node is
//     img + (total - stat) from its column.
//
// Scope (host: tcol_candidate): N32 ranges, the compact Fit /
// BalancedAllocation profile, every weighted total < 2^14, no carried slots.
// Results equal the slot walk's (and the oracle's) bit for bit.

constexpr int kTcMask = (1 << 14) - 1;

// col word: stat | total << 14 | held max taint << 28 | held max affinity << 29 | p1 feasible << 30 | live << 31
__device__ __forceinline__ uint32_t tc_word(int32_t stat, int32_t total, bool ft, bool fa, bool p1f, bool live) {
  return ((uint32_t)stat & kTcMask) | (((uint32_t)total & kTcMask) << 14) | (ft ? 1u << 28 : 0u) |
         (fa ? 1u << 29 : 0u) | (p1f ? 1u << 30 : 0u) | (live ? 1u << 31 : 0u);
}
__device__ __forceinline__ uint64_t tc_key(uint32_t w, int node) {
  return (w >> 31) ? argmax_key((int64_t)((w >> 14) & kTcMask), node) : 0;
}


// The compact Fit / BalancedAllocation profile as plain scalars (member selects
// on a struct in registers can turn into scratch address selects).
struct TcProf {
  bool least;
  int32_t wc, wm;
  float i_ws, i_wc, i_wm;
};
__device__ __forceinline__ TcProf tc_prof(const CmProf& m) {
  return TcProf{m.least, (int32_t)m.wc, (int32_t)m.wm, m.inv_ws, m.inv_wc, m.inv_wm};
}

// One pod's values for the column evaluation (a lane holds P of them).
struct TcPod {
  int64_t req[4];          // NodeResourcesFit filter columns
  int32_t rc, rm;          // requested cpu milli / memory MiB (BalancedAllocation)
  int32_t nzc, nzm;        // non-zero cpu milli / memory MiB (Fit score)
  int64_t rm64, nzm64;     // MW: memory in bytes
  int32_t wfit, wba;       // weights if the plugin scores this pod, else 0
  int32_t mt, ma;          // phase-1 maxima of the raw TaintToleration / NodeAffinity scores
  uint32_t mask;           // bits 0-3: Fit filter checks column r; bit 4: Fit filter on
  int32_t wt, wa;          // TaintToleration / NodeAffinity weights if scored, else 0 (spec walk)
  float inv_mt, inv_ma;    // qdiv32 estimates of 1 / mt, 1 / ma
};

// Pod k's batch-uniform values for the decision, the assume and its result:
// one LDS record per pod, read a step ahead.
struct TcU {
  int64_t req[4];          // assume deltas of the requested columns (0 beyond R)
  int64_t nzc, nzm;        // non-zero deltas
  int32_t nfeas, K, ht, ha;
  uint32_t flags;          // bit 0 phase-1 range error, 1 TaintToleration scores, 2 NodeAffinity scores, 3 commit
  uint32_t st_pf, st_sc;   // result status bits: always / when scored
  uint32_t skip, skip_sc;  // result score_skip: unscored / scored
  int32_t pad[3];
};
static_assert(sizeof(TcU) % 16 == 0, "LDS record");

// A live row's values, uniform across the wave (the node just assumed onto).
struct TcRow {
  int64_t fr[4];           // allocatable - requested per column
  int32_t pods, allowed;
  int32_t ac, am, sac, sam, qc0, qm0, nc0, nm0;
  int64_t am64, sam64, qm064, nm064;   // MW: memory in bytes
  bool hc, hm;
  float ic, im, iws;
  int32_t ws;
  double rcpc, rcpm;
};

// MW (the wide-memory instance): memory stays in int64 bytes (quantities not
// whole MiB, e.g. kubelet Ki values, or past the N32 ranges; ksg_range32 mw
// bounds them below 2^46): Fit's memory quotient is qdiv (64-bit dividend,
// float estimate, one correction), BalancedAllocation's fraction ddiv_r of
// the byte values with ddiv_rcp of the byte allocatable.  Both equal the int64
// forms bit for bit (a quotient of equally scaled integers is unchanged), so
// the walk's decisions equal the N32 ones wherever both apply.
template <bool MW = false>
__device__ __forceinline__ TcRow tc_row(const TcProf& m, const int64_t (&w)[SlotLayout<4>::W]) {
  using SL = SlotLayout<4>;
  TcRow r;
#pragma unroll
  for (int c = 0; c < 4; c++) r.fr[c] = w[2 * c] - w[2 * c + 1];
  r.pods = (int32_t)w[SL::PODS];
  r.allowed = (int32_t)w[SL::ALLOWED];
  r.ac = (int32_t)w[2 * KSG_RES_CPU];
  r.hc = r.ac > 0;
  r.sac = r.hc ? r.ac : 1;
  r.ic = __int_as_float((int32_t)w[SL::INVC]);
  r.qc0 = (int32_t)w[SL::NZC];
  r.nc0 = (int32_t)w[2 * KSG_RES_CPU + 1];
  r.rcpc = __longlong_as_double(w[SL::DAC]);
  if constexpr (MW) {
    r.am64 = w[2 * KSG_RES_MEM];
    r.hm = r.am64 > 0;
    r.sam64 = r.hm ? r.am64 : 1;
    r.im = __builtin_amdgcn_rcpf((float)r.sam64);
    r.rcpm = ddiv_rcp((double)r.sam64);
    r.qm064 = w[SL::NZM];
    r.nm064 = w[2 * KSG_RES_MEM + 1];
    r.am = r.sam = r.qm0 = r.nm0 = 0;
  } else {
    r.am = (int32_t)(w[2 * KSG_RES_MEM] >> 20);
    r.hm = r.am > 0;
    r.sam = r.hm ? r.am : 1;
    r.im = __int_as_float((int32_t)w[SL::INVM]);
    r.qm0 = (int32_t)(w[SL::NZM] >> 20);
    r.nm0 = (int32_t)(w[2 * KSG_RES_MEM + 1] >> 20);
    r.rcpm = __longlong_as_double(w[SL::DAM]);
    r.am64 = r.sam64 = r.qm064 = r.nm064 = 0;
  }
  r.ws = (r.hc ? m.wc : 0) + (r.hm ? m.wm : 0);
  float iws = __builtin_amdgcn_readfirstlane(0) ? 0.0f : m.i_wm;   // selects on values
  iws = r.hc ? m.i_wc : iws;
  iws = r.hc && r.hm ? m.i_ws : iws;
  r.iws = iws;
  return r;
}

// NodeResourcesFit filter + the weighted Fit / BalancedAllocation scores of a
// pod on a row: cm_scores32 with the row's parts hoisted (same operations, same
// order, same bits).
template <bool MW = false>
__device__ __forceinline__ bool tc_eval(const TcProf& m, const TcPod& h, const TcRow& r, int32_t& fb) {
  bool fits = r.pods + 1 <= r.allowed;
#pragma unroll
  for (int c = 0; c < 4; c++) fits = fits && (!((h.mask >> c) & 1u) || h.req[c] <= r.fr[c]);
  fits = fits || !((h.mask >> 4) & 1u);
  const int32_t qc = r.qc0 + h.nzc;
  int32_t xc, sm;
  double fm;
  if (m.least) xc = qc > r.ac ? 0 : (r.ac - qc) * 100;
  else xc = (qc > r.ac ? r.ac : qc) * 100;
  if constexpr (MW) {
    const int64_t qm = r.qm064 + h.nzm64;
    int64_t xm;
    if (m.least) xm = qm > r.am64 ? 0 : (r.am64 - qm) * 100;
    else xm = (qm > r.am64 ? r.am64 : qm) * 100;
    sm = (int32_t)qdiv(xm, r.sam64, r.im);
    fm = ddiv_r((double)(r.nm064 + h.rm64), (double)r.sam64, r.rcpm);
  } else {
    const int32_t qm = r.qm0 + h.nzm;
    int32_t xm;
    if (m.least) xm = qm > r.am ? 0 : (r.am - qm) * 100;
    else xm = (qm > r.am ? r.am : qm) * 100;
    sm = qdiv32(xm, r.sam, r.im);
    fm = ddiv_r((double)(r.nm0 + h.rm), (double)r.sam, r.rcpm);
  }
  const int32_t sc = qdiv32(xc, r.sac, r.ic);
  const int32_t num = (r.hc ? sc * m.wc : 0) + (r.hm ? sm * m.wm : 0);
  const int32_t fs = r.ws == 0 ? 0 : qdiv32(num, r.ws, r.iws);
  double fc = ddiv_r((double)(r.nc0 + h.rc), (double)r.sac, r.rcpc);
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = r.hc && r.hm ? fabs((fc - fm) / 2) : 0.0;
  const int32_t bs = (int32_t)((1 - sd) * (double)100);
  fb = fs * h.wfit + bs * h.wba;
  return fits;
}


// the column evaluation's values of one pod
__device__ __forceinline__ TcPod tc_pod(const ksg_pod& p, const ksg_profile& prof, const P1Stats& s1, bool fit_filter_on,
                                        int R) {
  TcPod h;
  uint32_t mk = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    h.req[r] = r < R ? p.req[r] : 0;
    const bool chk = r < R && h.req[r] > 0 && !(r >= 3 && ((prof.fit_ignored_res >> r) & 1u));
    mk |= chk ? 1u << r : 0u;
  }
  if (fit_filter_on && !((p.filter_skip >> KSG_PL_NODE_RESOURCES_FIT) & 1u)) mk |= 1u << 4;
  h.mask = mk;
  h.rc = (int32_t)p.req[KSG_RES_CPU];
  h.rm = (int32_t)(p.req[KSG_RES_MEM] >> 20);
  h.nzc = (int32_t)p.nz_cpu;
  h.nzm = (int32_t)(p.nz_mem >> 20);
  h.rm64 = p.req[KSG_RES_MEM];
  h.nzm64 = p.nz_mem;
  const uint32_t smask = prof.score_mask & ~p.score_skip;
  h.wfit = (smask & bit(KSG_PL_NODE_RESOURCES_FIT)) ? (int32_t)prof.weight[KSG_PL_NODE_RESOURCES_FIT] : 0;
  h.wba = (smask & bit(KSG_PL_BALANCED_ALLOCATION)) ? (int32_t)prof.weight[KSG_PL_BALANCED_ALLOCATION] : 0;
  h.mt = s1.mt;
  h.ma = s1.ma;
  h.wt = (smask & bit(KSG_PL_TAINT_TOLERATION)) ? (int32_t)prof.weight[KSG_PL_TAINT_TOLERATION] : 0;
  h.wa = (smask & bit(KSG_PL_NODE_AFFINITY)) ? (int32_t)prof.weight[KSG_PL_NODE_AFFINITY] : 0;
  h.inv_mt = s1.inv_mt;
  h.inv_ma = s1.inv_ma;
  return h;
}

// A pod's running maxima and counters over the columns carried in from the
// previous batch (two-batch window), written by ksg_tcol_carry.
struct TcInit {
  uint64_t b1, b2;
  int32_t s1, s2;
  uint32_t cnt;
  uint32_t pad;
};

// Two-batch window: the nodes the previous batch assumed onto (a.carry, its
// slot order) start this batch as columns.  Block q = pod q of the batch, lane
// t = carried node t (<= 64): pod q on node t's live row (global state after
// the previous walk), the column word into tc_colinit[t][q], and the pod's
// top-2 / counters over the carried columns into tc_init[q].  Same
// arithmetic as the walk's column evaluation.
template <int P>
__global__ __launch_bounds__(64) void ksg_tcol_carry(BatchArgs a) {
  constexpr int QS = 64 * P;
  __shared__ ksg_profile s_prof;
  const int q = blockIdx.x, lane = threadIdx.x;
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  for (int i = lane; i < (int)(sizeof(ksg_profile) / 4); i += 64)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  __syncthreads();
  const ksg_profile& prof = s_prof;
  bool fit_filter_on = false;
  for (int kf = 0; kf < prof.n_filter; kf++) fit_filter_on |= prof.filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  const TcProf cm = tc_prof(cm_prof(prof));
  const int nc0 = *a.carry_n;
  const ksg_pod& p = a.pods[a.b0 + q];
  const P1Stats s1 = a.p1[q];
  const TcPod h = tc_pod(p, prof, s1, fit_filter_on, R);
  uint64_t key = 0;
  uint32_t dc = 0;
  if (lane < nc0) {
    const int d = a.carry[lane];
    int64_t w[SlotLayout<4>::W];
#pragma unroll
    for (int x = 0; x < SlotLayout<4>::W; x++)
      w[x] = slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, x, R, d), x, R);
    const TcRow row = tc_row(cm, w);
    const uint64_t x = a.rec[(size_t)q * N + d];
    const bool p1f = (x >> 63) != 0;
    const bool ft = p1f && (int32_t)((x >> 48) & 0xff) == h.mt;
    const bool fa = p1f && (int32_t)((x >> 32) & 0xffff) == h.ma;
    const int32_t stat = a.stat[(size_t)q * N + d];
    int32_t fb = 0;
    const bool live = tc_eval(cm, h, row, fb) && p1f;
    const int32_t total = stat + fb;
    a.tc_colinit[lane * QS + q] = tc_word(stat, total, ft, fa, p1f, live);
    key = live ? argmax_key(total, d) : 0;
    dc = (p1f ? 1u : 0u) + (live ? 1u << 8 : 0u) + (p1f && !live && ft ? 1u << 16 : 0u) +
         (p1f && !live && fa ? 1u << 24 : 0u);
  }
  // keys of distinct nodes are distinct: the top two and their slots
  const uint64_t b1 = wreduce(key, OpMaxU64{});
  const uint64_t m1 = __ballot(b1 != 0 && key == b1);
  const int s1i = m1 ? __builtin_ctzll(m1) : -1;
  const uint64_t k2 = lane == s1i ? 0 : key;
  const uint64_t b2 = wreduce(k2, OpMaxU64{});
  const uint64_t m2 = __ballot(b2 != 0 && k2 == b2);
  const uint32_t cn = wreduce(dc, OpAdd32{});
  if (lane == 0) {
    TcInit ti;
    ti.b1 = b1;
    ti.b2 = b2;
    ti.s1 = s1i;
    ti.s2 = m2 ? __builtin_ctzll(m2) : -1;
    ti.cnt = cn;
    ti.pad = 0;
    reinterpret_cast<TcInit*>(a.tc_init)[q] = ti;
  }
}

// Per-pod running maxima over the columns.
struct TcTop {
  uint64_t b1, b2;
  int32_t s1, s2;
  bool x2;       // b2 exact: the best over every column other than s1
  bool rescan;   // b1 unknown until the columns are rescanned
};
__device__ __forceinline__ void tc_top_init(TcTop& t) {
  t.b1 = t.b2 = 0;
  t.s1 = t.s2 = -1;
  t.x2 = true;
  t.rescan = false;
}
// Column s of this pod now holds key v; fresh: s was not a column before.
// Branch-free (each lane is a different pod):
//   s held b1:  v >= b2 (b2 exact): b1 = v; else b1 = b2 and b2 becomes a lower
//               bound (v); b2 inexact: rescan.
//   s held b2:  v > b1: swap in; v >= b2: b2 = v; else b2 = v, inexact.
//   otherwise:  v > b1: b2 = old b1, exact again; v > b2: b2 = v.
__device__ __forceinline__ void tc_top_update(TcTop& t, uint64_t v, int s, bool fresh) {
  const bool h1 = !fresh && s == t.s1;
  const bool h2 = !fresh && !h1 && t.x2 && s == t.s2;
  const bool gt1 = v > t.b1, ge2 = v >= t.b2, gt2 = v > t.b2;
  const uint64_t b1 = t.b1, b2 = t.b2;
  const int32_t s1 = t.s1, s2 = t.s2;
  // h1
  const bool h1_keep = t.x2 && ge2;           // b1 = v
  const bool h1_fall = t.x2 && !ge2;          // b1 = b2, s1 = s2, b2 = v, s2 = s, inexact
  // h2 / other: v above b1 takes the lead
  const bool lead = !h1 && gt1;
  uint64_t nb1 = b1, nb2 = b2;
  int32_t ns1 = s1, ns2 = s2;
  bool nx2 = t.x2, nrs = t.rescan;
  nb1 = h1 ? (h1_fall ? b2 : v) : (lead ? v : b1);
  ns1 = h1 ? (h1_fall ? s2 : s1) : (lead ? s : s1);
  nb2 = h1 ? (h1_fall ? v : b2) : lead ? b1 : (h2 || gt2) ? v : b2;
  ns2 = h1 ? (h1_fall ? s : s2) : lead ? s1 : (h2 || gt2) ? s : s2;
  nx2 = h1 ? (h1_fall ? false : t.x2) : lead ? (h2 ? t.x2 : true) : h2 ? ge2 : t.x2;
  nrs = nrs || (h1 && !t.x2);
  (void)h1_keep;
  t.b1 = nb1;
  t.b2 = nb2;
  t.s1 = ns1;
  t.s2 = ns2;
  t.x2 = nx2;
  t.rescan = nrs;
}

// the phase-1 records and statics of node e for this lane's pods, and node
// e's live columns (slot word `lane`), issued without waiting
template <int P>
struct TcFetch {
  uint64_t rec[P];
  int32_t stat[P];
  SlotFetch<4> col;
};
template <int P>
__device__ __forceinline__ TcFetch<P> tc_fetch(const BatchArgs& a, const SlotPlan& plan, int lane, int e) {
  TcFetch<P> f;
  // node-major copies: node e's values for every pod of the batch are contiguous
  const uint64_t* rt = a.rect + (size_t)e * (64 * P);
  const int32_t* st = a.statt + (size_t)e * (64 * P);
#pragma unroll
  for (int i = 0; i < P; i++) {
    f.rec[i] = rt[lane + 64 * i];
    f.stat[i] = st[lane + 64 * i];
  }
  f.col = slot_plan_fetch<4>(plan, e);
  return f;
}

// [nb][N] -> [N][qs] copies of the phase-1 records and the N32 statics (rows
// beyond nb are left as they are: the walk never reads them for a live pod).
// Tiles of 32 nodes through LDS: reads and writes are both contiguous.
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_batch_transpose(BatchArgs a) {
  __shared__ uint64_t s_r[128][33];
  __shared__ int32_t s_s[128][33];
  const int tid = threadIdx.x;
  const int N = a.c.N, nb = a.nb, qs = a.qs;
  const int n0 = blockIdx.x * 32;
  for (int x = tid; x < nb * 32; x += 256) {
    const int j = x >> 5, nn = x & 31, n = n0 + nn;
    if (n < N) {
      s_r[j][nn] = a.rec[(size_t)j * N + n];
      s_s[j][nn] = a.stat[(size_t)j * N + n];
    }
  }
  __syncthreads();
  for (int x = tid; x < 32 * qs; x += 256) {
    const int nn = x / qs, j = x - nn * qs, n = n0 + nn;
    if (n < N && j < nb) {
      a.rect[(size_t)n * qs + j] = s_r[j][nn];
      a.statt[(size_t)n * qs + j] = s_s[j][nn];
    }
  }
  if (a.tk_done) {   // the window's hand-off to the speculate-and-verify walk (as ksg_batch_topk's)
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      using G1 = __attribute__((address_space(1))) unsigned;
      const unsigned old = __hip_atomic_fetch_add((G1*)a.tk_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x - 1) {
        __hip_atomic_store((G1*)a.tk_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((G1*)a.tk_done, a.tk_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}
#endif  // KSG_PART

template <int P>
__global__ __launch_bounds__(64) void ksg_batch_phase2t(BatchArgs a) {
  using SL = SlotLayout<4>;
  constexpr int QS = 64 * P;   // column-store row length (pods)
  constexpr int SW = SL::W;
  static_assert(QS <= KSG_BATCH_MAX, "pods per batch");
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ int32_t s_clist[2 * QS];   // carried + this batch's slots
  __shared__ ksg_result s_res[QS];
  __shared__ __attribute__((aligned(16))) TcU s_u[QS];
  __shared__ uint8_t s_touched[2 * QS];   // two-batch window: slot assumed onto in this batch

  const int lane = threadIdx.x, tid = lane;
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  const int nb = a.nb;
  const int cm_words = (((N + 31) / 32) + 3) & ~3;
  constexpr int POD_WORDS = sizeof(ksg_pod) / 4;
  uint32_t* s_cmask = reinterpret_cast<uint32_t*>(s_dyn);
  ksg_pod* s_pods = reinterpret_cast<ksg_pod*>(s_dyn + cm_words);
  int32_t* s_prog = s_dyn + cm_words + nb * POD_WORDS;
  int64_t* s_slot = reinterpret_cast<int64_t*>(s_dyn + ((cm_words + nb * POD_WORDS + a.prog_len + 3) & ~3));
  const int nslots = nb + (a.carry ? a.k_extra : 0);   // carried (<= the previous batch) + this batch's
  uint32_t* s_col = reinterpret_cast<uint32_t*>(s_slot + (size_t)nslots * SL::STRIDE);

  for (int i = lane; i < cm_words; i += 64) s_cmask[i] = 0;
  for (int i = lane; i < nb * POD_WORDS; i += 64)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + a.b0)[i];
  for (int i = lane; i < a.prog_len; i += 64) s_prog[i] = a.prog[a.prog_lo + i];
  for (int i = lane; i < (int)(sizeof(ksg_profile) / 4); i += 64)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  __syncthreads();
  const ksg_profile& prof = s_prof;
  const TcProf cm = tc_prof(cm_prof(prof));
  const bool ipa_filter = ipa_in_filter(prof);
  const bool ipa_score = ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;
  const SlotPlan plan = slot_plan<4, true>(c, a.st, lane, R);
  auto changed = [&](int n) { return ((s_cmask[n >> 5] >> (n & 31)) & 1u) != 0; };

  // this lane's pods, and the per-pod uniform records
  TcPod hp[P];
  TcTop tp[P];
  uint32_t cnt[P];   // feasible at phase 1 | live << 8 | lost taint holders << 16 | lost affinity holders << 24
#pragma unroll
  for (int i = 0; i < P; i++) {
    const int q = lane + 64 * i;
    const int qq = q < nb ? q : 0;
    const ksg_pod& p = s_pods[qq];
    const P1Stats s1 = a.p1[qq];
    hp[i] = tc_pod(p, prof, s1, fit_filter_on, R);
    const uint32_t smask = prof.score_mask & ~p.score_skip;
    tc_top_init(tp[i]);
    cnt[i] = 0;
    if (a.carry && q < nb) {   // the previous batch's columns (ksg_tcol_carry)
      const TcInit ti = reinterpret_cast<const TcInit*>(a.tc_init)[q];
      tp[i].b1 = ti.b1;
      tp[i].b2 = ti.b2;
      tp[i].s1 = ti.s1;
      tp[i].s2 = ti.s2;
      cnt[i] = ti.cnt;
    }
    if (q < nb) {
      TcU u;
#pragma unroll
      for (int r = 0; r < 4; r++) u.req[r] = r < R ? p.req[r] : 0;
      u.nzc = p.nz_cpu;
      u.nzm = p.nz_mem;
      u.nfeas = s1.nfeas;
      u.K = s1.K;
      u.ht = s1.ht;
      u.ha = s1.ha;
      const bool wt = (smask & bit(KSG_PL_TAINT_TOLERATION)) && prof.weight[KSG_PL_TAINT_TOLERATION];
      const bool wa = (smask & bit(KSG_PL_NODE_AFFINITY)) && prof.weight[KSG_PL_NODE_AFFINITY];
      u.flags = (s1.err ? 1u : 0u) | (wt ? 2u : 0u) | (wa ? 4u : 0u) | (p.commit >= 0 ? 8u : 0u);
      const bool ipa_none = p.ipa < 0;
      const bool ps_skip = ipa_none && ipa_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u);
      u.st_pf = ipa_none && ipa_filter ? KSG_ST_IPA_PREFILTER_SKIP : 0u;
      u.st_sc = KSG_ST_SCORED | (ps_skip ? KSG_ST_IPA_PRESCORE_SKIP : 0u);
      u.skip = p.score_skip;
      u.skip_sc = p.score_skip | (ps_skip ? bit(KSG_PL_INTER_POD_AFFINITY) : 0u);
      u.pad[0] = u.pad[1] = u.pad[2] = 0;
      s_u[q] = u;
    }
  }
  __syncthreads();

  int nc = 0;   // |D|, uniform
  if (a.carry) {   // the previous batch's nodes: live rows, columns from ksg_tcol_carry
    nc = *a.carry_n;
    for (int t = lane; t < nc * SW; t += 64) {
      const int i = t / SW, w = t - i * SW;
      s_slot[(size_t)i * SL::STRIDE + w] = slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, w, R, a.carry[i]), w, R);
    }
    for (int t = lane; t < nc; t += 64) {
      const int d = a.carry[t];
      s_clist[t] = d;
      atomicOr(&s_cmask[d >> 5], 1u << (d & 31));
    }
    for (int x = lane; x < nc * QS; x += 64) s_col[x] = a.tc_colinit[x];
  }
  for (int t = lane; t < 2 * QS; t += 64) s_touched[t] = 0;
  __syncthreads();
  // Loop-carried loads are double-buffered (A/B by step parity, the loop
  // unrolled by two): a register copy of a load still in flight would wait
  // for it.  T_{k+1} is loaded a step ahead; T_0's first entry is pod 0's best node.
  uint64_t tA = nb > 1 ? a.top[(size_t)KSG_BATCH_MAX + lane] : 0;   // T_1
  uint64_t tB = 0;
  uint64_t bu = 0;
  bool bu_full = false;
  {
    const uint64_t t0 = a.top[lane];
    const int K0 = s_u[0].K;
    const uint64_t m = __ballot(lane < K0 && !changed(key_node(t0)));
    bu = m ? readlane64(t0, __builtin_ctzll(m)) : 0;
    bu_full = m == 0 && K0 > 64;
  }
  int spec = bu ? key_node(bu) : -1;
  TcFetch<P> fA = tc_fetch<P>(a, plan, lane, spec >= 0 ? spec : 0);
  TcFetch<P> fB = fA;

#ifdef KSG_STAMPS
  unsigned long long st_acc[16] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif
  (void)tid;
  // one step: decide pod k, assume it, prefetch for pod k + 1 into (tnext, fnext),
  // evaluate the new column for the pods after k
  // pod k's record is read a step ahead (double-buffered like the loads)
  TcU uA = s_u[0], uB = uA;
  // T_{k+1}'s changed flags, a step ahead (pA: T_1 against the carried nodes)
  bool pA = false, pB = false;
  {
    const int t1 = key_node(tA);
    pA = changed((unsigned)t1 < (unsigned)N ? t1 : 0);
  }
  int prev_sel = -1;
  auto step = [&](const int k, uint64_t& tcur, uint64_t& tnext, TcFetch<P>& fc, TcFetch<P>& fnext, const TcU& u,
                  TcU& unext, const bool pcur, bool& pnext) {
    KSG_STAMP(0);
    const int ki = k >> 6, kl = k & 63;
    const bool more = k + 1 < nb;
    unext = s_u[more ? k + 1 : k];
    const int K1 = more ? unext.K : 0;
    const uint64_t t64a = tcur;
    // T_{k+2}, consumed at the top of the next step (vmcnt counts in issue
    // order: node spec's values, issued at the end of this step, come after it)
    // (unconditional, clamped: a load issued on one path only makes the
    // compiler's vmcnt path-dependent, i.e. vmcnt(0) at the next wait)
    tnext = a.top[(size_t)min(k + 2, nb - 1) * KSG_BATCH_MAX + lane];
    // flags of T_{k+1} against D before this pod (LDS reads overlap the decision)
    const int tn = key_node(t64a);
    // T_{k+1}'s changed flags against D before pod k - 1 were read at the end of
    // the previous step (pcur); pods k - 1 and k are added below
    const bool pre_chg = lane >= K1 || pcur || tn == prev_sel;
    // ---- decide pod k ---------------------------------------------------------
    // lazy rescan: pod k's best column is unknown (rare)
    {
      const bool need = __builtin_amdgcn_readlane((int)(P > 1 && ki ? tp[P - 1].rescan : tp[0].rescan), kl) != 0;
      if (need) {   // every flagged pod of the wave at once
        bool rs[P];
#pragma unroll
        for (int i = 0; i < P; i++) {
          rs[i] = tp[i].rescan;
          if (rs[i]) tc_top_init(tp[i]);
        }
        for (int t = 0; t < nc; t++) {
          const int nd = s_clist[t];
#pragma unroll
          for (int i = 0; i < P; i++) {
            const uint64_t v = tc_key(s_col[t * QS + lane + 64 * i], nd);
            TcTop x = tp[i];
            tc_top_update(x, v, t, true);
            if (rs[i]) tp[i] = x;
          }
        }
      }
    }
    KSG_STAMP(1);
    // pod k's lane values (selects on values: a runtime index into the
    // register arrays would put them in scratch)
    const bool hi = P > 1 && ki;
    const uint64_t k0 = readlane64(hi ? tp[P - 1].b1 : tp[0].b1, kl);
    const int32_t kidx = __builtin_amdgcn_readlane(hi ? tp[P - 1].s1 : tp[0].s1, kl);
    const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)(hi ? cnt[P - 1] : cnt[0]), kl);
    const int feas1 = kc & 0xff, live_n = (kc >> 8) & 0xff, lost_t = (kc >> 16) & 0xff, lost_a = kc >> 24;
    if (bu_full) {   // every one of T_k's first 64 entries is changed: the rest of T_k (rare)
      uint64_t best = 0;
      for (int b = 0; b < u.K; b += 64) {
        uint64_t tkey = 0;
        if (b + lane < u.K) {
          const uint64_t key = a.top[(size_t)k * KSG_BATCH_MAX + b + lane];
          if (!changed(key_node(key))) tkey = key;
        }
        best = max(best, wreduce(tkey, OpMaxU64{}));
      }
      bu = best;
    }
    const int unch = u.nfeas - feas1;
    int nfeas = unch + live_n;
    const bool renorm = nfeas >= 2 && ((u.flags & 1u) || ((u.flags & 2u) && u.ht - lost_t <= 0) ||
                                       ((u.flags & 4u) && u.ha - lost_a <= 0));
    int selected = -1, idx = -1;
    uint32_t status = 0;
    if (renorm) {
      const ksg_pod& p = s_pods[k];
      const PodView v = make_view(c, prof, p, s_prog + (p.blob - a.prog_lo), a.prog);
      const uint64_t* rec = a.rec + (size_t)k * N;
      const int32_t* img = a.img + (size_t)k * N;
      // live record of pod k on changed slot t: img + (total - stat) with the phase-1 raw scores
      auto live_rec = [&](int t) -> uint64_t {
        const uint32_t w = s_col[t * QS + k];
        if (!(w >> 31)) return 0;
        const int nd = s_clist[t];
        const uint64_t x = rec[nd];
        const int64_t part = (int64_t)img[nd] + (int64_t)((w >> 14) & kTcMask) - (int64_t)(w & kTcMask);
        return pack_rec(part, (x >> 48) & 0xff, (x >> 32) & 0xffff);
      };
      Red r{0, 0, 0, 0x7fffffff};
      for (int n = lane; n < N; n += 64) {
        if (changed(n)) continue;
        const uint64_t x = rec[n];
        if (!(x >> 63)) continue;
        r.nfeas += 1;
        r.max_t = max(r.max_t, (int64_t)((x >> 48) & 0xff));
        r.max_a = max(r.max_a, (int64_t)((x >> 32) & 0xffff));
      }
      for (int t = lane; t < nc; t += 64) {
        const uint64_t x = live_rec(t);
        if (!(x >> 63)) continue;
        r.nfeas += 1;
        r.max_t = max(r.max_t, (int64_t)((x >> 48) & 0xff));
        r.max_a = max(r.max_a, (int64_t)((x >> 32) & 0xffff));
      }
      const int64_t max_t = wreduce(r.max_t, OpMax64{}), max_a = wreduce(r.max_a, OpMax64{});
      nfeas = (int)wreduce((uint32_t)r.nfeas, OpAdd32{});
      uint64_t best = 0;
      uint32_t err = 0;
      auto visit = [&](uint64_t x, int n) {
        const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
        const uint64_t key = argmax_key(total_score(v, part, rt, ra, max_t, max_a, err, nullptr, nullptr), n);
        best = key > best ? key : best;
      };
      for (int n = lane; n < N; n += 64) {
        if (changed(n)) continue;
        const uint64_t x = rec[n];
        if (x >> 63) visit(x, n);
      }
      for (int t = lane; t < nc; t += 64) {
        const uint64_t x = live_rec(t);
        if (x >> 63) visit(x, s_clist[t]);
      }
      best = wreduce(best, OpMaxU64{});
      err = wreduce(err, OpOr32{});
      status |= KSG_ST_SCORED;
      if (err) status |= KSG_ST_SCORE_ERROR;
      else selected = key_node(best);
      if (selected >= 0 && changed(selected)) {
        for (int b = 0; b < nc && idx < 0; b += 64) {
          const uint64_t mk = __ballot(b + lane < nc && s_clist[b + lane] == selected);
          if (mk) idx = b + __builtin_ctzll(mk);
        }
      }
    } else if (nfeas == 1) {
      if (unch == 1) {
        selected = key_node(bu);
      } else {   // the one live column
        selected = key_node(k0);
        idx = kidx;
      }
    } else if (nfeas >= 2) {
      status |= KSG_ST_SCORED;
      if (bu > k0) {
        selected = key_node(bu);
      } else {
        selected = key_node(k0);
        idx = kidx;
      }
    }
    const bool added = selected >= 0 && idx < 0;
    const int slot = added ? nc : idx;
    KSG_STAMP(2);

    // ---- assume pod k onto `selected` -------------------------------------------
    // this lane's word of the assume (row word `lane` += delta)
    // (selects, not u.req[lane-dependent index]: that would put u in scratch)
    const int rl = (lane >> 1) & 3;
    const int64_t req_l = rl == 0 ? u.req[0] : rl == 1 ? u.req[1] : rl == 2 ? u.req[2] : u.req[3];
    const int64_t row_delta = lane < 8 ? ((lane & 1) ? req_l : 0)
                              : lane == SL::NZC ? u.nzc
                              : lane == SL::NZM ? u.nzm
                              : lane == SL::PODS ? 1 : 0;
    if (added && selected != spec) fc = tc_fetch<P>(a, plan, lane, selected);   // dependent loads (rare)
    if (selected >= 0) {
      if (lane == 0) s_touched[slot] = 1;
      int64_t* row = s_slot + (size_t)slot * SL::STRIDE;
      if (added) {
        const int64_t col_val = slot_word_value<4, true>(fc.col, lane, R);
        if (lane < SW) row[lane] = col_val + row_delta;
        if (lane == 0) {
          atomicOr(&s_cmask[selected >> 5], 1u << (selected & 31));
          s_clist[nc] = selected;
        }
      } else if (lane < SW) {
        row[lane] += row_delta;
      }
      if ((u.flags & 8u) && lane == 0) {   // PodTopologySpread / InterPodAffinity count tables
        const ksg_pod& p = s_pods[k];
        const int32_t* cw = s_prog + (p.commit - a.prog_lo);
        const int ns = *cw++;
        for (int i = 0; i < ns; i++) a.st.cnt[(size_t)cw[i] * N + selected] += 1;
        cw += ns;
        const int nt = *cw++;
        for (int i = 0; i < nt; i++) {
          const int t = cw[2 * i];
          const uint32_t lv = c.label_val[(size_t)c.tmpl_col[t] * N + selected];
          if (!lv) continue;
          a.st.tab[c.tmpl_off[t] + lv] += c.tmpl_kind[t] == KSG_TMPL_PREF ? cw[2 * i + 1] : 1;
          a.st.tmpl_total[t] += 1;
        }
      }
    }
    if (lane == 0) {
      const bool sc = (status & KSG_ST_SCORED) != 0;
      ksg_result res;
      res.selected = selected;
      res.n_feasible = nfeas;
      res.status = status | u.st_pf | (sc ? u.st_sc : 0u);
      res.score_skip = sc ? u.skip_sc : u.skip;
      s_res[k] = res;
    }
    nc += added ? 1 : 0;
    KSG_STAMP(3);

    // ---- pod k + 1's best unchanged node and its loads; the next records -------
    {   // (issued on every step, see tnext)
      const bool tf = !more || pre_chg || tn == selected;
      const uint64_t m = __ballot(!tf);
      bu = m ? readlane64(t64a, __builtin_ctzll(m)) : 0;
      bu_full = more && m == 0 && K1 > 64;
      spec = bu ? key_node(bu) : -1;
      fnext = tc_fetch<P>(a, plan, lane, spec >= 0 ? spec : 0);
    }
    KSG_STAMP(4);
    // ---- the column of `selected` for pods q > k ------------------------------
    if (selected >= 0 && more) {
      int64_t w[SW];
      {
        const int4* src = reinterpret_cast<const int4*>(s_slot + (size_t)slot * SL::STRIDE);
#pragma unroll
        for (int x = 0; x < SW / 2; x++) reinterpret_cast<int4*>(w)[x] = src[x];
      }
      const TcRow row = tc_row(cm, w);
      KSG_STAMP(5);
#pragma unroll
      for (int i = 0; i < P; i++) {
        if (k >= 64 * (i + 1) - 1) continue;   // every pod of this register set is decided (uniform)
        const int q = lane + 64 * i;
        const bool act = q > k && q < nb;
        uint32_t old = 0;
        int32_t stat;
        bool p1f, ft, fa;
        if (added) {
          const uint64_t x = fc.rec[i];
          p1f = (x >> 63) != 0;
          ft = p1f && (int32_t)((x >> 48) & 0xff) == hp[i].mt;
          fa = p1f && (int32_t)((x >> 32) & 0xffff) == hp[i].ma;
          stat = fc.stat[i];
        } else {
          old = s_col[slot * QS + q];
          p1f = (old >> 30) & 1u;
          ft = (old >> 28) & 1u;
          fa = (old >> 29) & 1u;
          stat = (int32_t)(old & kTcMask);
        }
        int32_t fb = 0;
        const bool live = tc_eval(cm, hp[i], row, fb) && p1f;
        const int32_t total = stat + fb;
        const uint32_t wd = tc_word(stat, total, ft, fa, p1f, live);
        if (act) s_col[slot * QS + q] = wd;
        const uint32_t dc = added ? (p1f ? 1u : 0u) + (live ? 1u << 8 : 0u) + (p1f && !live && ft ? 1u << 16 : 0u) +
                                        (p1f && !live && fa ? 1u << 24 : 0u)
                          : ((old >> 31) && !live) ? (ft ? 1u << 16 : 0u) + (fa ? 1u << 24 : 0u) - (1u << 8) : 0u;
        cnt[i] += act ? dc : 0u;
        TcTop x = tp[i];
        tc_top_update(x, live ? argmax_key(total, selected) : 0, slot, added);
        if (act) tp[i] = x;
      }
    }
    {   // T_{k+2}'s changed flags against D up to this pod (LDS, used two steps on)
      const int t2 = key_node(tnext);
      pnext = changed((unsigned)t2 < (unsigned)N ? t2 : 0);
    }
    prev_sel = selected;
    KSG_STAMP(6);

  };
  for (int k = 0; k < nb; k += 2) {
    step(k, tA, tB, fA, fB, uA, uB, pA, pB);
    if (k + 1 < nb) step(k + 1, tB, tA, fB, fA, uB, uA, pB, pA);
  }
#ifdef KSG_STAMPS
  if (lane == 0 && a.stamps)
    for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], st_acc[i]);
#endif
  __syncthreads();
  // rows and results go out once, after the walk
  for (int i = lane; i < nc * SW; i += 64) {
    const int sl = i / SW, w = i - sl * SW, node = s_clist[sl];
    const int64_t val = s_slot[(size_t)sl * SL::STRIDE + w];
    if (w < 8 && (w & 1) && (w >> 1) < R) a.st.requested[(size_t)(w >> 1) * N + node] = val;
    else if (w == SL::NZC || w == SL::NZM) a.st.nonzero[(size_t)(w - SL::NZC) * N + node] = val;
    else if (w == SL::PODS) a.st.pod_count[node] = (int32_t)val;
  }
  for (int i = lane; i < nb; i += 64) {
    a.placements[a.out0 + i] = s_res[i].selected;
    if (a.results) a.results[a.out0 + i] = s_res[i];
  }
  for (int i = lane; i < 2 * nb; i += 64) a.pmax[i] = 0;   // ready for the next batch's phase 1
  if (a.carry_out) {   // the nodes this batch touched, in slot order, for the next batch
    int base = 0;
    for (int b = 0; b < nc; b += 64) {
      const bool t = b + lane < nc && s_touched[b + lane];
      const uint64_t m = __ballot(t);
      if (t) a.carry_out[base + __popcll(m & ((1ull << lane) - 1))] = s_clist[b + lane];
      base += __popcll(m);
    }
    if (lane == 0) *a.carry_out_n = base;
  }
}
