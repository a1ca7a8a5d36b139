// Single-replica queue with PodTopologySpread / InterPodAffinity across the
// whole chip (config 3), included by ksched.hip inside its anonymous namespace.
//
// ksg_queue_topo_kernel walks every node of a pod four times from ONE
// workgroup; at 15,000 nodes that is ~30 dependent node visits per lane per
// sweep, 1.2 ms per pod.  Here G co-resident workgroups share each pod: lane
// (wg, tid) owns nodes (k * G + wg) * 256 + tid, k < KN, for the whole queue,
// so a node's mutable columns (requested, non-zero, pod count, selector
// counts) are only ever read and written by one lane.
//
// The queue runs in batches of kCoopBatch pods.  Per batch, ksg_sweep_static
// first computes every (pod, node)'s replica-independent plugin results
// (NodeUnschedulable, NodeName, TaintToleration, NodeAffinity verdicts, raw
// taint / node-affinity / image scores) in one massively parallel launch, so
// the per-pod critical path below reads one 8-byte record per node instead of
// walking taint, toleration, image and requirement lists.  Then
// ksg_topo_coop<KN> walks the batch; per pod:
//
//   setup      every workgroup stages the pod and lays out its LDS histograms
//   phase 1    pre-pass over the lane's nodes: per-domain counts into the LDS
//              histograms; the workgroup publishes its partial histogram and
//              partial scalars in its own slot (plain stores, no contention)
//   -- grid barrier --
//   phase 2    every workgroup folds the G partial slots into its LDS copy;
//              sweep A (filters incl. PTS/IPA, node-local scores), the IPA raw
//              score and, with one soft PTS constraint, the extremes of its
//              per-node count; partial reductions into the slot
//   -- grid barrier --  (+ one more for >= 2 soft PTS constraints: their raw
//                         scores' min/max)
//   phase 3    fold the phase-2 partials; normalise, weight, argmax
//   -- grid barrier --
//   phase 4    fold the argmax partials; the owner lane of the selected node
//              assumes the pod (node columns, selector counts; domain tables
//              by atomics); workgroup 0 writes the result
//
// With one soft constraint the PodTopologySpread raw score of a node is
// round(m * w + maxSkew - 1) for a node with the topology key (0 without it),
// m its domain count and w = log(size + 2) > 0, which is monotone in m: the
// min / max over the feasible nodes follow from the min / max of m, so the
// sizes and the min / max need no extra barrier.
//
// Partial slots are rewritten in full every pod, and each is read only between
// the barrier after its write and the next write (always two barriers later),
// so one set suffices.  A pod whose histograms exceed the partial-slot budget
// merges them with atomics into an accumulator set instead (two sets by pod
// parity; workgroup 0 resets the set of pod j - 1 in phase 2 of pod j).
// Grid barrier: a monotonic arrival counter; every storing wave drains its
// stores, one lane releases (agent scope), arrives, polls relaxed with
// s_sleep, and acquires (agent scope); every cross-workgroup word is read with
// agent-scope atomic loads (MI355X guide, Guideline 16).  The poll is bounded:
// on timeout the kernel records an error and every workgroup leaves.

constexpr int kCoopBatch = 64;      // pods per launch (static records [kCoopBatch][N])
constexpr int kCoopPHist = 512;     // partial-histogram words per workgroup slot
constexpr int kCoopLabCols = 16;    // KN == 1: label columns of the lane's node staged in LDS
constexpr int kCoopTmpl = 2048;     // term templates whose column / table offset are staged in LDS
constexpr int kCoopLog = 512;       // log_table entries staged in LDS

struct CoopPart {   // one workgroup's partial results of the current pod
  // phase 1
  long long hard_min[kMaxHard];
  int32_t hard_dom[kMaxHard];
  long long soft_empty[kMaxSoft];
  long long aff_total;
  int32_t pref_any;
  // phase 2
  int32_t nfeas, minidx, n_ignored, has_val, has_zero;
  int32_t soft_present[kMaxSoft], soft_seen[kMaxSoft];
  long long max_t, max_a, mmin, mmax, imin, imax;
  // phase 2b (>= 2 soft constraints)
  long long pmin, pmax;
  // phase 3
  unsigned long long best;
  int32_t err;
  // the pod's lag selectors' counts at this workgroup's best-key node and at
  // its lowest feasible node (the winner's become the lag delta's old counts)
  int32_t best_cnt[kLagSel], min_cnt[kLagSel];
};

struct CoopAcc {    // atomics fallback for large histograms
  int32_t hist[KSG_HIST_MAX];
};


// gld / gst / gadd / gor and arrive_and_wait_sc1: ksched_sweep.h

#ifdef KSG_STAMPS
#define KSG_CSTAMP(seg)                                                     \
  do {                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                      \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();             \
    if (tid == 0 && wg == 0) { st_acc[seg] += _t - st_last; st_last = _t; } \
    __builtin_amdgcn_sched_barrier(0);                                      \
  } while (0)
#else
#define KSG_CSTAMP(seg) do {} while (0)
#endif

struct CoopArgs {
  DevCluster c;
  DevState st;
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* profile;
  int32_t first, count, G;     // pods [first, first + count): one batch
  int32_t out0;                // output index of pod `first`
  int32_t* placements;
  ksg_result* results;         // or null
  const uint64_t* srec;        // [count][N] static records of the batch
  CoopPart* parts;             // [G]
  int32_t* phist;              // [G][kCoopPHist]
  CoopAcc* acc;                // [2], zeroed before the launch
  unsigned* bar;               // per-workgroup barrier flags [G][32] (one 128-B line each), zeroed before the launch
  unsigned* timeout;           // set when a barrier poll gave up
  int32_t pmode;               // 1: partial-slot histograms folded by every workgroup; 0: atomics into acc
  unsigned long long* stamps;  // diagnostic build only (KSG_STAMPS): per-segment cycle sums
  int32_t commit;              // 0: evaluate only (ksg_eval / ksg_eval_view): no assume
  // capture (CAP instances): every pod's status words and the profile's score
  // rows, compact (row q = plugin cap_rows[q], the normalising ones first),
  // every node written (no memset): [count][N] / [count][rows][N]
  uint32_t* cap_fs;
  char* cap_raw;
  char* cap_norm;              // rows q < cap_n_normrows
  char* cap_tot;
  int32_t cap_rows[KSG_NPLUGINS];
  int32_t cap_n_rows, cap_n_normrows, cap_narrow;
  // CAP == 2, the per-cycle host block (one pod): the result, then the flag
  ksg_result* h_res;
  unsigned* h_flag;
  unsigned seq;
  // the maintained domain tables (ksched_topo_tables.h)
  TopoTables tt;
  int32_t use_tables;          // 1: pods within their scope skip phase 1 and barrier 1
  int32_t tables_inkernel;     // 1 (the per-cycle tables): elig and the fill tasks of each pod computed at
                               // its setup (tables_fill) instead of read from tt.elig / tt.fo
  unsigned gen;                // barrier flag generation: flags are (gen << 16) + epoch, monotonic across
                               // launches, so nothing is reset per launch
  int32_t fused_static;        // 1 (one pod): every lane computes its node's static record itself
                               // (no ksg_sweep_static launch)
  int32_t cap_es;              // CAP == 2: bytes per row value (2, 4, 8); a value that does not fit
                               // sets *h_ovf and the host evaluates again wider
  unsigned* h_ovf;
  ksg_pod* wpods;              // CAP == 2, a staged append read in place (pods / prog point into the
                               // staging buffer): workgroup 0 copies it here (pod `first`) ...
  int32_t* wprog;              // ... and its programs here; null: none
  const int32_t* sprog;
  int64_t slen;
  unsigned* arrive;            // CAP == 2: the completion counter (never reset between launches: the last
                               // of each launch's G arrivals stores the result; zeroed with the flags)
                               // CAP == 3: one per window row, 32 words apart
  // CAP == 3, a window of the speculative topology queue (ksched_topo_win.h):
  // grid (G, kmax); row y evaluates pod *win_cursor + y against the state the
  // window starts from, with its own barrier flags / partial slots / atomics
  // set (bar, parts, phist, acc offset by the row), and stores, instead of
  // selecting and assuming, its nodes' static totals, its G tiles' best keys
  // and the pod's facts for ksg_topo_walk
  const int32_t* win_cursor;   // the run's first undecided pod (ksg_topo_walk advances it)
  const int32_t* win_len;      // [pods of the run]: the window starting at that pod
  int32_t win_base, win_end;   // the run's pods [win_base, win_end)
  int32_t win_kmax;            // rows of the grid (gridDim.y)
  int32_t* win_tot;            // [kmax][N]
  unsigned long long* win_top; // [kmax][G][kmax]
  WinPod* win_pod;             // [kmax]
  unsigned* win_done;          // arrivals of the launch's workgroups (the last walks the window and zeroes it)
  unsigned long long* win_stats;   // [3] windows, pods decided, windows ended early
};

// Hand-offs between the G workgroups without cache maintenance (MI355X guide,
// Guideline 16, "Valid forms" table row 1): every byte another workgroup
// reads is stored with an agent-scope (sc1, write-through) store or an
// agent-scope atomic and read with an agent-scope global (sc1) load, every
// storing wave drains its stores before the workgroup barrier in front of the
// arrival, one lane per workgroup adds to the counter and polls it with sc1
// loads, the other waves load after the workgroup barrier that lane joins.
// No release (buffer_wbl2) and no acquire (buffer_inv): the round-1 barrier
// paid both, ~8-9 k cycles each (profiles/r1/stamps_topo_coop.txt).
// Grid barrier on per-workgroup flags: each workgroup's lane 0 stores the
// epoch into its own 128-byte line (sc1, after every wave's drain and the
// workgroup barrier), and wave 0 polls all G flags with one sc1 load per lane
// (G <= 256).  No atomic on a shared counter: 59 workgroups adding to one
// word serialise at the memory side (the guide's "Valid forms" row 1, sharded).
__device__ __forceinline__ bool coop_barrier(unsigned* flags, unsigned* timeout, int G, unsigned& epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 stores and atomics are done
  __syncthreads();
  epoch += 1;
  __shared__ int s_to;
  const int tid = threadIdx.x;
  if (tid < 64) {
    if (tid == 0) gst(&flags[(size_t)blockIdx.x * 32], epoch);
    unsigned spins = 0;
    int to = 0;
    for (;;) {
      bool ok = true;
      for (int l = tid; l < G; l += 64) ok = ok && gld(&flags[(size_t)l * 32]) >= epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 26) || gld(timeout)) {
        if (tid == 0) gst(timeout, 1u);
        to = 1;
        break;
      }
    }
    if (tid == 0) s_to = to;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler ordering only: loads stay below the poll
  __syncthreads();
  return s_to == 0;
}

// PodTopologySpread with one soft constraint: the per-node count m of
// pts_score_node (same branches), or ignored / no key.  0: m valid, 1: the
// node lacks the key (score 0), 2: ignored node (score -1).
__device__ __forceinline__ int pts_soft1_m(const DevCluster& c, const PodView& v, const TopoCtx& t, int n,
                                          int64_t& m) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  if (g.require_all && !has_all(c, g.soft, g.n_soft, 6, n)) return 2;
  const int32_t* sc = g.soft;
  const uint32_t val = lab(c, sc[0], n);
  if (!val) return 1;
  const Slot& sl = s.soft[0];
  if (sc[5]) m = cnt_at(t.cnt, c.N, sl.sel, n);
  else if (!sl.unique) m = t.hist[sl.hist + val];
  else if (val == 1) m = s.soft_empty[0];
  else m = inclusion(c, v, t, sc[3], sc[4], n) ? cnt_at(t.cnt, c.N, sl.sel, n) : 0;
  return 0;
}

__device__ __forceinline__ int64_t pts_soft1_score(const TopoProg& g, const TopoShared& s, int64_t m) {
  const double x = (double)m * s.soft_w[0];
  double score = 0.0;
  score += x + (double)(g.soft[2] - 1);
  return (int64_t)round(score);
}

// eval_node_src with the replica-independent plugins read from the node's
// static record (t.rec): RunFilterPlugins (feasibility; the coop path records
// no per-node status word) + the raw scores.
__device__ __forceinline__ NodeEval eval_node_rec(const DevCluster& c, const ksg_profile& prof, const PodView& v,
                                                  const NodeCols& L, int n, const TopoCtx& t, const CmProf& cm) {
  const ksg_pod& p = *v.p;
  const uint64_t sr = t.rec;
  NodeEval e{0, 0, 0, 0, 0};
  uint32_t st = 0;
  if (sr & kSrNotEval) {
    st = KSG_FS_NOT_EVALUATED;
  } else {
    for (int kf = 0; kf < prof.n_filter && !st; kf++) {
      const int pl = prof.filter_order[kf];
      if ((v.fskip >> pl) & 1u) continue;
      switch (pl) {
        case KSG_PL_NODE_UNSCHEDULABLE:
          if (sr & kSrUnsched) st = pl + 1;
          break;
        case KSG_PL_NODE_NAME:
          if (sr & kSrNodeName) st = pl + 1;
          break;
        case KSG_PL_TAINT_TOLERATION:   // payload: the node's first untolerated taint slot (static record)
          if (sr & kSrTaint) st = (uint32_t)(pl + 1) | ((uint32_t)((sr >> kSrTaintSlotShift) & 0xffff) << 8);
          break;
        case KSG_PL_NODE_AFFINITY:
          if (sr & kSrNodeAff) st = (uint32_t)(pl + 1) | (1u << 8);
          break;
        case KSG_PL_NODE_RESOURCES_FIT: {
          const uint32_t b = fit_filter(c, p, L, prof.fit_ignored_res);
          if (b) st = (uint32_t)(pl + 1) | (b << 8);
          break;
        }
        case KSG_PL_POD_TOPOLOGY_SPREAD:
          if (t.g->pts_filter) {
            const uint32_t r = pts_filter_node(c, v, t, n);
            if (r) st = (uint32_t)(pl + 1) | (r << 8);
          }
          break;
        case KSG_PL_INTER_POD_AFFINITY:
          if (t.g->ipa) {
            const uint32_t r = ipa_filter_node(c, t, n);
            if (r) st = (uint32_t)(pl + 1) | (r << 8);
          }
          break;
        default:
          break;
      }
    }
  }
  e.st = st;
  if (st != 0) return e;
  if (cm.fast && (v.smask & (bit(KSG_PL_NODE_RESOURCES_FIT) | bit(KSG_PL_BALANCED_ALLOCATION)))) {
    int64_t sf, sb;   // both chains at once (fit_ba_cm: the same bits)
    fit_ba_cm(cm, p, L, sf, sb);
    if (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) e.part += sf * v.w_fit;
    if (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) e.part += sb * v.w_ba;
  } else {
    if (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) e.part += fit_score(prof, p, L) * v.w_fit;
    if (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) e.part += ba_score(prof, p, L) * v.w_ba;
  }
  if (v.smask & bit(KSG_PL_IMAGE_LOCALITY)) {
    e.img = (int64_t)((sr >> 32) & 0xff) * v.w_img;
    e.part += e.img;
  }
  if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) e.rt = (int64_t)((sr >> 8) & 0xff);
  if (v.smask & bit(KSG_PL_NODE_AFFINITY)) e.ra = (int64_t)((sr >> 16) & 0xffff);
  return e;
}

// NodeInfo.AddPod for node n by the lane that owns it: node columns and
// selector counts with plain stores, domain tables with atomics.
// tab_now = false: the template tables reach tab one pod late (the lag buffer,
// applied by workgroup 0; readers add it meanwhile).
__device__ __forceinline__ void coop_commit(const DevCluster& c, const DevState& st, const ksg_pod& p,
                                            const int32_t* commit_prog, int n, bool tab_now = true) {
  const int N = c.N;
  for (int r = 0; r < c.R; r++) st.requested[(size_t)r * N + n] += p.req[r];
  st.nonzero[n] += p.nz_cpu;
  st.nonzero[(size_t)N + n] += p.nz_mem;
  st.pod_count[n] += 1;
  if (commit_prog) {
    const int32_t* w = commit_prog;
    const int ns = *w++;
    for (int i = 0; i < ns; i++) st.cnt[(size_t)w[i] * N + n] += 1;
    w += ns;
    const int nt = *w++;
    for (int i = 0; tab_now && i < nt; i++) {
      const int t = w[2 * i];
      const uint32_t val = c.label_val[(size_t)c.tmpl_col[t] * N + n];
      if (!val) continue;
      gadd(st.tab + c.tmpl_off[t] + val, c.tmpl_kind[t] == KSG_TMPL_PREF ? w[2 * i + 1] : 1);
      gadd(st.tmpl_total + t, 1);
    }
  }
}

// Workgroup 0 applies a pending assume to the tables (dom, tot, cc) and, when
// they were lagged, to the template tables.  Called between the barrier after
// every reader of the tables of this pod and the next barrier.  Every update
// is an independent no-return atomic: wave 0 lane i takes selector i's
// (column, table) pairs, wave 1 the template entries, wave 2 tot and cc.
__device__ __forceinline__ void lag_apply(const DevCluster& cg, const DevState& st, const TopoTables& t,
                                          const LagDelta& d, bool tables, bool tab) {
  const int tid = threadIdx.x, N = cg.N;
  if (d.node < 0) return;
  if (tables && tid < d.n_sel) {   // wave 0: the domain tables of selector tid
    const int s = d.sel[tid];
    const int b = t.sp_off[s], e = t.sp_off[s + 1];
    for (int k = b; k < e; k++) {
      const int col = t.sp[2 * k], off = t.sp[2 * k + 1];
      const uint32_t v = cg.label_val[(size_t)col * N + d.node];
      if (v) gadd(t.dom + off + v, 1);
    }
  }
  if (tables && tid >= 128 && tid < 128 + d.n_sel) {   // wave 2: totals and count-of-counts
    const int i = tid - 128, s = d.sel[i];
    gadd(t.tot + s, 1);
    const int co = t.cc_off[s];
    if (co >= 0) {
      const int k = d.old_cnt[i];
      if (k + 1 >= t.Kc - 1) {
        __hip_atomic_store((__attribute__((address_space(1))) unsigned*)t.invalid, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      } else {
        gadd(t.cc + co + k, -1);
        gadd(t.cc + co + k + 1, 1);
      }
    }
  }
  if (tab && tid >= 64 && tid < 64 + d.n_tmpl) {   // wave 1: the template-table entries
    const int i = tid - 64;
    if (d.tidx[i] >= 0) {
      gadd(st.tab + d.tidx[i], d.tw[i]);
      gadd(st.tmpl_total + d.tt[i], 1);
    }
  }
}

struct OpMinL { __device__ long long operator()(long long a, long long b) const { return a < b ? a : b; } };
struct OpMaxL { __device__ long long operator()(long long a, long long b) const { return a > b ? a : b; } };
struct OpAddL { __device__ long long operator()(long long a, long long b) const { return a + b; } };
struct OpAddI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a + b; } };
struct OpMinI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a < b ? a : b; } };
struct OpOrI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a | b; } };

// LL: the host guarantees KN == 1, every label column, the column vocabulary
// and every term template fit their LDS copies; the evaluators' tables are then
// LDS pointers at compile time (ds_read, not flat loads on the node paths).
// CAP: 0 placement only; 1 capture into device rows (captured queues);
// 2 capture into the pinned host block + completion flag (the per-cycle
// evaluation of a topology pod: one pod, a.commit = 0).
template <int KN, bool LL = false, int CAP = 0>
__global__ __launch_bounds__(256) void ksg_topo_coop(CoopArgs a) {
  constexpr int BLOCK = 256, NW = BLOCK / 64;
  constexpr long long BIG = 0x7fffffffffffffffll;
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ __attribute__((aligned(16))) int32_t s_hist[KSG_HIST_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ TopoProg s_g;
  __shared__ TopoShared s_t;
  __shared__ long long s_l[NW][16];
  __shared__ int32_t s_i[NW][16];
  __shared__ int s_size[kMaxSoft];
  __shared__ long long s_tt[4];
  __shared__ uint8_t s_wkind[kCoopPHist];   // partial-slot word: 1 histogram count (add), 0 presence bits (or), 2 mark (skip)
  // read-only node / template tables staged once per launch: every label,
  // column and template lookup of the per-pod critical path is an LDS read
  __shared__ uint32_t s_lab[kCoopLabCols * BLOCK];
  __shared__ int32_t s_cv[kCoopLabCols];
  __shared__ uint8_t s_cu[kCoopLabCols];
  __shared__ int32_t s_tcol[kCoopTmpl], s_toff[kCoopTmpl];
  __shared__ ksg_pod s_pods[kCoopBatch];   // the batch's pod records
  __shared__ double s_log[kCoopLog];       // log_table[0 .. kCoopLog): topologyNormalizingWeight of small domains
  // the one-pod lag (ksched_topo_tables.h): the previous pod's assume, not yet
  // in the tables / template tables; identical in every workgroup
  __shared__ LagDelta s_lag;
  __shared__ int s_lag_tab;      // 1: s_lag's template-table entries are pending (readers add them)
  __shared__ int s_prev_imm;     // the previous pod wrote its template tables at once: barrier 1 orders them
  __shared__ int s_tables_ok;    // the tables are exact for this launch
  __shared__ int s_last;         // CAP == 2: this workgroup arrived last (stores the result)
  __shared__ int s_lsel[kLagSel];   // this pod's matched selectors (commit program) ...
  __shared__ int s_nlsel;           // ... and their number (may exceed kLagSel)
  __shared__ int s_wmin;            // this workgroup's lowest feasible node (phase 2)
  __shared__ unsigned long long s_wbest;   // this workgroup's best key (phase 3)
  __shared__ unsigned long long s_wtop[NW];   // CAP == 3: the tile's best keys, one round at a time
  __shared__ uint8_t s_elig[kCoopBatch];    // tables_scope of the batch's pods
  __shared__ int s_inv;                     // the tables were invalidated (read per pod)
  __shared__ int4 s_fo[kTopoFill];          // the pod's fill tasks (tables' fo), loaded at setup
  __shared__ long long s_totv[1 + kMaxPref];   // tot[sel_all], tot[pref selectors], loaded at setup

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wg = blockIdx.x, G = a.G;
  const DevCluster& cg = a.c;   // global tables (assume writes; other nodes' labels)
  const int N = cg.N;
  const DevState& st = a.st;
  const TopoTables& tt = a.tt;
  // the pods of this launch: [first, first + count); CAP == 3 reads them from
  // the window cursor, and row blockIdx.y takes pod first + blockIdx.y alone
  static_assert(CAP != 3 || KN == 1, "window rows: one node per lane");
  int first = a.first, count = a.count, kq_lo = 0;
  if constexpr (CAP == 3) {
    first = *a.win_cursor;
    if (first >= a.win_end) return;
    count = min(min(a.win_len[first - a.win_base], (int)gridDim.y), a.win_end - first);
    kq_lo = (int)blockIdx.y;
    if (kq_lo >= count) return;
  }
  const int kq_hi = CAP == 3 ? kq_lo + 1 : count;
  const int row = CAP == 3 ? kq_lo : 0;   // this row's flags, partial slots and atomics set
  CoopPart* const parts = a.parts + (size_t)row * G;
  int32_t* const phist = a.phist + (size_t)row * G * kCoopPHist;
  CoopAcc* const accs = a.acc + 2 * row;
  unsigned* const rbar = a.bar + (size_t)row * G * 32;   // this row's barrier flags
  if (tid == 0) {
    s_lag.node = -1;
    s_lag.n_sel = s_lag.n_tmpl = 0;
    s_lag_tab = 0;
    s_prev_imm = 0;
    s_tables_ok = a.use_tables && !gld(tt.invalid);
  }
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.profile)[i_];
  for (int i = tid; i < count * (int)(sizeof(ksg_pod) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + first)[i];
  if (!a.tables_inkernel)
    for (int i = tid; i < count; i += BLOCK) s_elig[i] = a.use_tables ? tt.elig[first - tt.first + i] : 0;
  if (CAP == 2 && a.wpods && wg == 0) {   // the staged append to the device pool (read by later launches)
    for (int i = tid; i < (int)(sizeof(ksg_pod) / 4); i += BLOCK)
      reinterpret_cast<int32_t*>(a.wpods)[i] = reinterpret_cast<const int32_t*>(a.pods + first)[i];
    for (int64_t i = tid; i < a.slen; i += BLOCK) a.wprog[i] = a.sprog[i];
  }
  const bool lab_lds = LL || (KN == 1 && cg.L <= kCoopLabCols);
  const bool col_lds = LL || cg.L <= kCoopLabCols;
  const bool tmpl_lds = LL || cg.n_tmpl <= kCoopTmpl;
  if (lab_lds) {
    const int n = wg * BLOCK + tid;
    for (int col = 0; col < cg.L; col++) s_lab[col * BLOCK + tid] = n < N ? cg.label_val[(size_t)col * N + n] : 0u;
  }
  if (col_lds && tid < cg.L) { s_cv[tid] = cg.col_vocab[tid]; s_cu[tid] = cg.col_unique[tid]; }
  if (tmpl_lds)
    for (int i = tid; i < cg.n_tmpl; i += BLOCK) { s_tcol[i] = cg.tmpl_col[i]; s_toff[i] = cg.tmpl_off[i]; }
  for (int i = tid; i < kCoopLog && i < cg.log_n; i += BLOCK) s_log[i] = cg.log_table[i];
  // KN == 1: the lane's node's Fit / BalancedAllocation columns stay in
  // registers for the launch (only this lane reads or assumes onto the node)
  NodeCols Lreg;
  if (KN == 1) {
    const int n = wg * BLOCK + tid;
    if (n < N) load_cols(cg, st.requested, st.nonzero, st.pod_count, n, Lreg);
  }
  __syncthreads();
  DevCluster cl = cg;   // the evaluators' view: the staged copies where they fit
  if (LL) {
    cl.label_val = s_lab; cl.lab_stride = BLOCK; cl.lab_base = wg * BLOCK;
    cl.col_vocab = s_cv; cl.col_unique = s_cu;
    cl.tmpl_col = s_tcol; cl.tmpl_off = s_toff;
  } else {
    if (lab_lds) { cl.label_val = s_lab; cl.lab_stride = BLOCK; cl.lab_base = wg * BLOCK; }
    if (col_lds) { cl.col_vocab = s_cv; cl.col_unique = s_cu; }
    if (tmpl_lds) { cl.tmpl_col = s_tcol; cl.tmpl_off = s_toff; }
  }
  const DevCluster& c = cl;
  const ksg_profile& prof = s_prof;
  const CmProf cmp = cm_prof(prof);   // Fit + BalancedAllocation over exactly {cpu, memory}: fit_ba_cm
  bool ipa_in_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_in_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  const bool ipa_in_score = (prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u;
  unsigned target = a.gen << 16;   // this launch's barrier epochs
  int prev_fallback_words = 0;   // words of the previous pod's atomics-merged histograms (0: partial slots)
  CoopPart* const mine = parts + wg;
  int32_t* const myhist = phist + (size_t)wg * kCoopPHist;
#ifdef KSG_STAMPS
  unsigned long long st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
                     st_last = __builtin_amdgcn_s_memtime();
#endif

  auto node_of = [&](int k) { return (k * G + wg) * BLOCK + tid; };
  // LDS words [base, base + nw) += (or |=) the same words of every workgroup's
  // partial slot: (word, workgroup) pairs over the lanes, four loads in flight
  auto fold_words = [&](int base, int nw, bool bits) {
    const int total = nw * G;
    for (int x0 = tid; x0 < total; x0 += 4 * BLOCK) {
      int32_t y[4];
      int w[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int x = x0 + u * BLOCK;
        w[u] = x / G;
        const int qg = x - w[u] * G;
        y[u] = x < total ? gld(phist + (size_t)qg * kCoopPHist + base + w[u]) : 0;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (!y[u]) continue;
        if (bits) atomicOr((uint32_t*)&s_hist[base + w[u]], (uint32_t)y[u]);
        else atomicAdd(&s_hist[base + w[u]], y[u]);
      }
    }
  };
  // LDS words [0, nw) of the histogram slots += / |= every workgroup's partial
  // slot, all at once: lanes walk (workgroup, word) with the word fastest, so a
  // wave reads 64 consecutive words of one partial; 8 loads in flight per lane
  auto fold_all = [&](int nw) {
    const int total = nw * G;
    for (int x0 = tid; x0 < total; x0 += 8 * BLOCK) {
      int32_t y[8];
      int w[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int x = x0 + u * BLOCK;
        const int qg = x / nw;
        w[u] = x - qg * nw;
        y[u] = x < total && s_wkind[w[u]] != 2 ? gld(phist + (size_t)qg * kCoopPHist + w[u]) : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (!y[u]) continue;
        if (s_wkind[w[u]]) atomicAdd(&s_hist[w[u]], y[u]);
        else atomicOr((uint32_t*)&s_hist[w[u]], (uint32_t)y[u]);
      }
    }
  };
  // block-wide fold of one value per lane: DPP within waves, partials in LDS
  auto bfold_l = [&](long long x, auto op, int slot) {
    x = wreduce(x, op);
    if (lane == 0) s_l[wv][slot] = x;
  };
  auto bfold_i = [&](int32_t x, auto op, int slot) {
    x = wreduce(x, op);
    if (lane == 0) s_i[wv][slot] = x;
  };
  auto get_l = [&](int slot, auto op) {
    long long x = s_l[0][slot];
    for (int i = 1; i < NW; i++) x = op(x, s_l[i][slot]);
    return x;
  };
  auto get_i = [&](int slot, auto op) {
    int32_t x = s_i[0][slot];
    for (int i = 1; i < NW; i++) x = op(x, s_i[i][slot]);
    return x;
  };

  constexpr int kCoopPrefetch = 4;   // program words per lane prefetched for the next pod
  int32_t nb[kCoopPrefetch] = {0, 0, 0, 0};
  int nb_len = 0;
  for (int kq = kq_lo; kq < kq_hi; kq++) {
    CoopAcc* acc = accs + (kq & 1);
    CoopAcc* nxt = accs + ((kq + 1) & 1);
    const uint64_t* srow = a.srec + (size_t)kq * N;
    __syncthreads();
    if (tid < (int)(sizeof(ksg_pod) / 4))
      reinterpret_cast<int32_t*>(&s_pod)[tid] = reinterpret_cast<const int32_t*>(&s_pods[kq])[tid];
    if (tid == BLOCK - 1) s_inv = s_tables_ok ? gld(tt.invalid) != 0 : 1;   // read beside the pod's staging
    if (kq == kq_lo || nb_len > kCoopPrefetch * BLOCK) {   // (CAP 3: each row's first and only pod)
      const int boff = s_pods[kq].blob, blen = s_pods[kq].blob_len;
      for (int i = tid; i < blen; i += BLOCK) s_blob[i] = a.prog[boff + i];
    } else {   // prefetched during the previous pod's last barrier
#pragma unroll
      for (int u = 0; u < kCoopPrefetch; u++)
        if (tid + u * BLOCK < nb_len) s_blob[tid + u * BLOCK] = nb[u];
    }
    __syncthreads();
    KSG_CSTAMP(15);   // (stamps build: the pod staged; segment 15 is phase 1's node loop otherwise)
    const ksg_pod& p = s_pod;
    if (tid == 64) {   // this pod's matched selectors (its commit program): the lag delta of its assume
      int nl = 0;
      if (p.commit >= 0) {
        const int32_t* cw = s_blob + (p.commit - p.blob);
        nl = cw[0];
        for (int i = 0; i < kLagSel && i < cw[0]; i++) s_lsel[i] = cw[1 + i];
      }
      s_nlsel = nl;
    }
    if (tid == 128) {   // the per-pod accumulators (beside tid 0's parse: other fields of s_t)
      for (int i = 0; i < kMaxHard; i++) { s_t.hard_min[i] = BIG; s_t.hard_dom[i] = 0; }
      for (int i = 0; i < kMaxSoft; i++) {
        s_t.soft_empty[i] = 0; s_t.soft_present[i] = 0; s_t.soft_empty_seen[i] = 0; s_size[i] = 0;
      }
      s_t.n_ignored = 0;
      s_t.aff_total = 0;
      s_t.pref_any = 0;
      s_tt[0] = s_tt[1] = s_tt[2] = 0;
    }
    if (tid == 0) {
      const PodView v0 = make_view(c, prof, p, s_blob, a.prog, true);
      parse_topo(p, s_blob, v0.fskip, v0.smask, s_g);
      layout_slots(c, s_g, s_t);
      // Tables scope (tables_scope, one flag per pod computed at the run's
      // start), the tables exact (no count-of-counts overflow in the previous
      // pod's lag_apply: s_inv) and the histograms within their limits.
    }
    // the per-cycle tables: this pod's scope and fill tasks, from its LDS
    // program beside tid 0's parse (another wave)
    if (a.tables_inkernel && tid == 192)
      s_elig[kq] = s_tables_ok && tables_fill(c, tt, p, s_blob, s_fo, p.blob) ? 1 : 0;
    uint64_t srk[KN];
    if (a.fused_static) {   // one pod: the record of ksg_sweep_static, computed in place
      const PodView vs = make_view(c, prof, s_pod, s_blob, a.prog);
#pragma unroll
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        srk[k] = n < N ? static_record(cg, s_pod, vs, n, cg.taint_effect) : 0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        srk[k] = srow[n < N ? n : 0];
      }
    }
    __syncthreads();
    KSG_CSTAMP(2);    // (stamps build: tid 0's parse and layout; segment 2 is barrier 1 otherwise)
    const bool ok = s_t.ok;
    const int words = ok ? s_t.words : 0;
    // this pod skips phase 1 and barrier 1: it reads the tables (their scope,
    // exact), or has nothing to count
    const bool pre_skip = !s_prev_imm && (!(ok && (s_g.pts_filter || s_g.pts_score || s_g.ipa)) ||
                                        (s_tables_ok != 0 && ok && s_elig[kq] && !s_inv));
    // a pod reading the tables: its fill tasks, the totals its affinity /
    // preferred terms read and the existing pods' template totals, loaded now
    // (every write they see is lagged or was applied before barrier 3 of the
    // previous pod), in flight through the rest of the setup
    const bool tab_read = pre_skip && s_tables_ok && ok;
    if (tab_read) {
      const TopoProg& g1 = s_g;
      if (tid < kTopoFill && !a.tables_inkernel) s_fo[tid] = tt.fo[(size_t)(first - tt.first + kq) * kTopoFill + tid];
      if (g1.ipa && tid >= 64 && tid < 64 + 1 + g1.n_pref) {
        const int sel = tid == 64 ? g1.sel_all : g1.pref[3 * (tid - 65) + 1];
        s_totv[tid - 64] = sel >= 0 ? (long long)gld(tt.tot + sel) : 0;
      }
      const int n_t = g1.ipa ? g1.n_ma + g1.n_mh + g1.n_mp : 0;
      for (int i = tid - 128; i >= 0 && i < n_t; i += BLOCK - 128) {
        const int which = i < g1.n_ma ? 0 : (i < g1.n_ma + g1.n_mh ? 1 : 2);
        const int tm = which == 0 ? g1.m_anti[i] : (which == 1 ? g1.m_hard[i - g1.n_ma] : g1.m_pref[i - g1.n_ma - g1.n_mh]);
        int32_t x = gld(&st.tmpl_total[tm]);
        if (s_lag_tab && s_lag.node >= 0)   // the previous pod's pending template entries
          for (int j = 0; j < s_lag.n_tmpl; j++) x += s_lag.tt[j] == tm && s_lag.tidx[j] >= 0 ? 1 : 0;
        if (x) atomicAdd((unsigned long long*)&s_tt[which], (unsigned long long)x);
      }
    }
    const bool pmode = a.pmode && words <= kCoopPHist && words * G <= 32768;
    for (int i = tid; i < words; i += BLOCK) s_hist[i] = 0;
    if (pmode && !pre_skip) {   // word kinds of the partial slot (fold_all, phase 1's hand-off)
      for (int w = tid; w < words; w += BLOCK) {
        int kind = 0;
        auto in = [&](const Slot& sl) {
          if (sl.unique) return;
          if (w >= sl.hist && w < sl.hist + sl.V) kind = 1;
          if (sl.mark >= 0 && w >= sl.mark && w < sl.mark + (sl.V + 31) / 32) kind = 2;
        };
        for (int i = 0; i < s_g.n_hard; i++) in(s_t.hard[i]);
        for (int i = 0; i < s_g.n_soft; i++) in(s_t.soft[i]);
        for (int i = 0; i < s_g.n_aff; i++) in(s_t.aff[i]);
        for (int i = 0; i < s_g.n_anti; i++) in(s_t.anti[i]);
        for (int i = 0; i < s_g.n_pref; i++) in(s_t.pref[i]);
        s_wkind[w] = (uint8_t)kind;
      }
    }
    PodView v = make_view(c, prof, p, s_blob, a.prog, true);
    const TopoProg& g = s_g;
    TopoCtx tc{&s_g, &s_t, s_hist, st.cnt, st.tab, true, false, 0};
    if (s_lag_tab && s_lag.node >= 0) {   // tab lags the previous pod's assume: readers add its entries
      tc.lag_idx = s_lag.tidx;
      tc.lag_w = s_lag.tw;
      tc.lag_n = s_lag.n_tmpl;
    }
    __syncthreads();
    // which partial values this pod needs at all (pod-uniform): folds of the
    // others are skipped
    bool need_hmin = false, need_se = false;
    for (int i = 0; i < g.n_hard; i++) need_hmin |= s_t.hard[i].unique != 0;
    for (int i = 0; i < g.n_soft; i++) need_se |= s_t.soft[i].unique && !g.soft[6 * i + 5];
    const bool need_aff = g.ipa && g.n_aff > 0, need_pref = g.ipa && g.n_pref > 0;
    KSG_CSTAMP(0);

    // ---- phase 1: pre-pass over this lane's nodes -------------------------
    // (skipped with the tables: the domain counts come from them in phase 2,
    // and barrier 1 is not needed either, every cross-workgroup write of the
    // previous pod being lagged)
    const bool pre = ok && (g.pts_filter || g.pts_score || g.ipa);
    const bool skip = pre_skip != 0;
    if (pre && !skip) {
      long long lmin[kMaxHard], ldom[kMaxHard], lempty[kMaxSoft], laff = 0, lany = 0;
#pragma unroll
      for (int i = 0; i < kMaxHard; i++) { lmin[i] = BIG; ldom[i] = 0; }
#pragma unroll
      for (int i = 0; i < kMaxSoft; i++) lempty[i] = 0;
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N) break;
        TopoCtx tn = tc;
        tn.has_rec = true;
        tn.rec = srk[k];
        if (g.pts_filter && has_all(c, g.hard, g.n_hard, 7, n)) {
#pragma unroll
          for (int i = 0; i < kMaxHard; i++) {
            if (i >= g.n_hard) break;
            const int32_t* h = g.hard + 7 * i;
            if (!inclusion(c, v, tn, h[5], h[6], n)) continue;
            const Slot& sl = s_t.hard[i];
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
            if (sl.unique) {
              lmin[i] = min(lmin[i], (long long)x);
              ldom[i] += 1;
            } else {
              const uint32_t val = lab(c, sl.col, n);
              atomicAdd(&s_hist[sl.hist + val], x);
              atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
            }
          }
        }
        if (g.pts_score && (!g.require_all || has_all(c, g.soft, g.n_soft, 6, n))) {
#pragma unroll
          for (int i = 0; i < kMaxSoft; i++) {
            if (i >= g.n_soft) break;
            const int32_t* sc = g.soft + 6 * i;
            if (sc[5] || !inclusion(c, v, tn, sc[3], sc[4], n)) continue;
            const Slot& sl = s_t.soft[i];
            uint32_t val = lab(c, sl.col, n);
            if (!val) val = 1;   // node.Labels[key] of a missing key is ""
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
            if (sl.unique) {
              if (val == 1) lempty[i] += x;
            } else {
              atomicAdd(&s_hist[sl.hist + val], x);
            }
          }
        }
        if (g.ipa) {
          if (g.n_aff > 0) {
            const int32_t x = cnt_at(st.cnt, N, g.sel_all, n);
            for (int i = 0; i < g.n_aff; i++) {
              const Slot& sl = s_t.aff[i];
              const uint32_t val = lab(c, sl.col, n);
              if (!val) continue;
              laff += x;
              if (!sl.unique) {
                atomicAdd(&s_hist[sl.hist + val], x);
                atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
              }
            }
          }
          for (int i = 0; i < g.n_anti; i++) {
            const Slot& sl = s_t.anti[i];
            const uint32_t val = lab(c, sl.col, n);
            if (!val || sl.unique) continue;
            atomicAdd(&s_hist[sl.hist + val], cnt_at(st.cnt, N, sl.sel, n));
            atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
          }
          for (int i = 0; i < g.n_pref; i++) {
            const Slot& sl = s_t.pref[i];
            const uint32_t val = lab(c, sl.col, n);
            if (!val) continue;
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
            lany |= x > 0;
            if (!sl.unique) {
              atomicAdd(&s_hist[sl.hist + val], x);
              atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
            }
          }
        }
      }
      KSG_CSTAMP(15);
      if (need_hmin) {
#pragma unroll
        for (int i = 0; i < kMaxHard; i++) {
          if (i >= g.n_hard) break;
          bfold_l(lmin[i], OpMinL{}, i);
          bfold_i((int32_t)ldom[i], OpAddI{}, 4 + i);
        }
      }
      if (need_se) {
#pragma unroll
        for (int i = 0; i < kMaxSoft; i++) {
          if (i >= g.n_soft) break;
          bfold_l(lempty[i], OpAddL{}, 8 + i);
        }
      }
      if (need_aff) bfold_l(laff, OpAddL{}, 12);
      if (need_pref) bfold_i((int32_t)lany, OpOrI{}, 13);
      __syncthreads();
      // publish this workgroup's partial
      if (pmode) {
        for (int i = tid; i < words; i += BLOCK) gst(&myhist[i], s_hist[i]);
      } else {
        auto merge_slot = [&](const Slot& sl) {
          if (sl.unique) return;
          for (int i = tid; i < sl.V; i += BLOCK)
            if (s_hist[sl.hist + i]) gadd(&acc->hist[sl.hist + i], s_hist[sl.hist + i]);
          const int bw = (sl.V + 31) / 32;
          for (int i = tid; i < bw; i += BLOCK)
            if (s_hist[sl.pres + i]) gor(&acc->hist[sl.pres + i], s_hist[sl.pres + i]);
        };
        for (int i = 0; i < g.n_hard; i++) merge_slot(s_t.hard[i]);
        for (int i = 0; i < g.n_soft; i++) merge_slot(s_t.soft[i]);
        for (int i = 0; i < g.n_aff; i++) merge_slot(s_t.aff[i]);
        for (int i = 0; i < g.n_anti; i++) merge_slot(s_t.anti[i]);
        for (int i = 0; i < g.n_pref; i++) merge_slot(s_t.pref[i]);
      }
      if (need_hmin && tid < g.n_hard) {
        gst(&mine->hard_min[tid], get_l(tid, OpMinL{}));
        gst(&mine->hard_dom[tid], get_i(4 + tid, OpAddI{}));
      } else if (need_se && tid >= 64 && tid < 64 + g.n_soft) {
        gst(&mine->soft_empty[tid - 64], get_l(8 + tid - 64, OpAddL{}));
      } else if (tid == 128) {
        if (need_aff) gst(&mine->aff_total, get_l(12, OpAddL{}));
        if (need_pref) gst(&mine->pref_any, get_i(13, OpOrI{}) != 0);
      }
    }
    KSG_CSTAMP(1);
    if (!skip && !coop_barrier(rbar, a.timeout, G, target)) return;
    KSG_CSTAMP(2);

    // ---- phase 2: fold the partials into LDS; sweep A --------------------------
    if (pre && skip) {
      // the domain counts from the tables, plus the pending assume of the
      // previous pod (s_lag: +1 on its node's domain for the selectors it matched)
      const LagDelta& d = s_lag;
      auto in_lag = [&](int sel) {
        int hit = -1;
        for (int i = 0; i < d.n_sel; i++) hit = d.sel[i] == sel ? i : hit;
        return d.node >= 0 ? hit : -1;
      };
      // the non-unique slots' histograms, task k = the k-th such slot in
      // layout order (s_fo: dom offset, presence offset, column, selector);
      // every load of a task (the table words, the lag node's label) in flight
      // at once
      int k_task = 0;
      auto fill = [&](const Slot& sl, bool pres) {   // hist (+ presence bits) of a non-unique slot
        const int4 f = s_fo[k_task++];
        const uint32_t lv = in_lag(sl.sel) >= 0 ? cg.label_val[(size_t)sl.col * N + d.node] : 0u;   // 0: none
        for (int v = tid; v < sl.V; v += BLOCK) s_hist[sl.hist + v] = gld(tt.dom + f.x + v) + (lv && (uint32_t)v == lv ? 1 : 0);
        if (pres)
          for (int w = tid; w < (sl.V + 31) / 32; w += BLOCK) s_hist[sl.pres + w] = (int32_t)tt.pres[f.y + w];
      };
      for (int i = 0; i < g.n_hard; i++)
        if (!s_t.hard[i].unique) fill(s_t.hard[i], true);
      for (int i = 0; i < g.n_soft; i++)
        if (!g.soft[6 * i + 5] && !s_t.soft[i].unique) fill(s_t.soft[i], false);
      if (g.ipa) {
        for (int i = 0; i < g.n_aff; i++)
          if (!s_t.aff[i].unique) fill(s_t.aff[i], true);
        for (int i = 0; i < g.n_anti; i++)
          if (!s_t.anti[i].unique) fill(s_t.anti[i], true);
        for (int i = 0; i < g.n_pref; i++)
          if (!s_t.pref[i].unique) fill(s_t.pref[i], true);
      }
      // unique hard keys: the minimum count over the nodes from the
      // count-of-counts table (constraint i on wave NW - 1 - i, off wave 0's fill loads)
      const int hw = NW - 1 - wv;
      if (hw < g.n_hard && s_t.hard[hw].unique) {
        const int sel = s_t.hard[hw].sel, co = tt.cc_off[sel], li = in_lag(sel);
        const int old = li >= 0 ? d.old_cnt[li] : -2;
        int first = 0x7fffffff;
        for (int k0 = 0; k0 < tt.Kc && first == 0x7fffffff; k0 += 64) {
          const int k = k0 + lane;
          const int x = k < tt.Kc ? gld(tt.cc + co + k) - (k == old ? 1 : 0) + (k == old + 1 ? 1 : 0) : 0;
          const unsigned long long b = __ballot(x > 0);
          if (b) first = k0 + __builtin_ctzll(b);
        }
        if (lane == 0) { s_t.hard_min[hw] = first; s_t.hard_dom[hw] = N; }
      }
      __syncthreads();
      if (tid == 0) {
        // the totals came with the setup (s_totv: tot[sel_all], tot[pref selector i])
        auto total = [&](int sel, long long t) { return t + (in_lag(sel) >= 0 ? 1 : 0); };
        for (int i = 0; i < g.n_soft; i++) s_t.soft_empty[i] = 0;   // no node lacks the key or has ""
        if (g.ipa) {
          long long af = 0;
          for (int i = 0; i < g.n_aff; i++) {
            const Slot& sl = s_t.aff[i];
            if (sl.unique) af += total(g.sel_all, s_totv[0]);
            else for (int v = 1; v < sl.V; v++) af += s_hist[sl.hist + v];
          }
          s_t.aff_total = af;
          int any = 0;
          for (int i = 0; i < g.n_pref; i++) {
            const Slot& sl = s_t.pref[i];
            if (sl.unique) any |= total(sl.sel, s_totv[1 + i]) > 0;
            else for (int v = 1; v < sl.V; v++) any |= s_hist[sl.hist + v] > 0;
          }
          s_t.pref_any = any;
        }
      }
      __syncthreads();
      for (int i = 0; i < g.n_hard; i++) {   // minimum over present domains of the non-unique hard slots
        const Slot& sl = s_t.hard[i];
        if (sl.unique) continue;
        long long m = BIG, dd = 0;
        for (int val = tid; val < sl.V; val += BLOCK)
          if (bit_get(s_hist, sl.pres, val)) { m = min(m, (long long)s_hist[sl.hist + val]); dd += 1; }
        m = wave_min64(m);
        dd = wave_sum64(dd);
        if (lane == 0) {
          atomicMin((unsigned long long*)&s_t.hard_min[i], (unsigned long long)m);
          atomicAdd(&s_t.hard_dom[i], (int)dd);
        }
      }
    } else if (pre) {
      if (pmode) {
        for (int i = tid; i < words; i += BLOCK) s_hist[i] = 0;
        __syncthreads();
        fold_all(words);   // counts add, presence bitmaps or, marks are left for phase 3
      } else {
        for (int i = tid; i < words; i += BLOCK) s_hist[i] = gld(&acc->hist[i]);
      }
      // scalars: lane q folds workgroup q's slot
      if (need_hmin || need_se || need_aff || need_pref) {
        long long hm[kMaxHard], se[kMaxSoft], af = 0;
        int32_t hd[kMaxHard], pa = 0;
#pragma unroll
        for (int i = 0; i < kMaxHard; i++) { hm[i] = BIG; hd[i] = 0; }
#pragma unroll
        for (int i = 0; i < kMaxSoft; i++) se[i] = 0;
        if (tid < G) {
          const CoopPart* q = parts + tid;
#pragma unroll
          for (int i = 0; i < kMaxHard; i++)
            if (need_hmin && i < g.n_hard) { hm[i] = gld(&q->hard_min[i]); hd[i] = gld(&q->hard_dom[i]); }
#pragma unroll
          for (int i = 0; i < kMaxSoft; i++)
            if (need_se && i < g.n_soft) se[i] = gld(&q->soft_empty[i]);
          if (need_aff) af = gld(&q->aff_total);
          if (need_pref) pa = gld(&q->pref_any);
        }
        __syncthreads();   // every wave is past its phase-1 get_*() reads
        if (need_hmin) {
#pragma unroll
          for (int i = 0; i < kMaxHard; i++) {
            if (i >= g.n_hard) break;
            bfold_l(hm[i], OpMinL{}, i);
            bfold_i(hd[i], OpAddI{}, 4 + i);
          }
        }
        if (need_se) {
#pragma unroll
          for (int i = 0; i < kMaxSoft; i++) {
            if (i >= g.n_soft) break;
            bfold_l(se[i], OpAddL{}, 8 + i);
          }
        }
        if (need_aff) bfold_l(af, OpAddL{}, 12);
        if (need_pref) bfold_i(pa, OpOrI{}, 13);
        __syncthreads();
        if (tid == 0) {
          if (need_hmin)
            for (int i = 0; i < g.n_hard; i++)
              if (s_t.hard[i].unique) {
                s_t.hard_min[i] = get_l(i, OpMinL{});
                s_t.hard_dom[i] = get_i(4 + i, OpAddI{});
              }
          if (need_se)
            for (int i = 0; i < g.n_soft; i++) s_t.soft_empty[i] = get_l(8 + i, OpAddL{});
          if (need_aff) s_t.aff_total = get_l(12, OpAddL{});
          if (need_pref) s_t.pref_any = get_i(13, OpOrI{}) != 0;
        }
        __syncthreads();
      }
      for (int i = 0; i < g.n_hard; i++) {   // minimum over present domains of the non-unique hard slots
        const Slot& sl = s_t.hard[i];
        if (sl.unique) continue;
        long long m = BIG, d = 0;
        for (int val = tid; val < sl.V; val += BLOCK)
          if (bit_get(s_hist, sl.pres, val)) { m = min(m, (long long)s_hist[sl.hist + val]); d += 1; }
        m = wave_min64(m);
        d = wave_sum64(d);
        if (lane == 0) {
          atomicMin((unsigned long long*)&s_t.hard_min[i], (unsigned long long)m);
          atomicAdd(&s_t.hard_dom[i], (int)d);
        }
      }
    }
    KSG_CSTAMP(3);
    if (wg == 0 && prev_fallback_words)   // the set of pod kq - 1, read by everyone by now
      for (int i = tid; i < prev_fallback_words; i += BLOCK) gst(&nxt->hist[i], 0);
    prev_fallback_words = pmode ? 0 : words;   // (a skipping pod still merges its soft marks into acc)
    if (!tab_read) {   // existing pods' terms matching this pod: totals, one template per lane (tab_read: setup)
      const int n_t = g.ipa ? g.n_ma + g.n_mh + g.n_mp : 0;
      for (int i = tid; i < n_t; i += BLOCK) {
        const int which = i < g.n_ma ? 0 : (i < g.n_ma + g.n_mh ? 1 : 2);
        const int tm = which == 0 ? g.m_anti[i] : (which == 1 ? g.m_hard[i - g.n_ma] : g.m_pref[i - g.n_ma - g.n_mh]);
        int32_t x = gld(&st.tmpl_total[tm]);
        if (s_lag_tab && s_lag.node >= 0)   // the previous pod's pending template entries
          for (int j = 0; j < s_lag.n_tmpl; j++) x += s_lag.tt[j] == tm && s_lag.tidx[j] >= 0 ? 1 : 0;
        if (x) atomicAdd((unsigned long long*)&s_tt[which], (unsigned long long)x);
      }
    }
    __syncthreads();
    if (tid == 0) {
      const long long ma = s_tt[0], mh = s_tt[1], mp = s_tt[2];
      s_t.ipa_skip_filter = !g.ipa || (ma == 0 && g.n_aff == 0 && g.n_anti == 0);
      s_t.ipa_skip_score = !g.ipa || !((prof.hard_pod_affinity_weight > 0 && mh > 0) || mp > 0);
      if (pre) {
        for (int i = 0; i < g.n_hard; i++)   // minMatchNum: 0 when fewer domains than minDomains
          if (s_t.hard_dom[i] < g.hard[7 * i + 3]) s_t.hard_min[i] = 0;
        if (s_t.pref_any) s_t.ipa_skip_score = 0;
      }
    }
    __syncthreads();
    KSG_CSTAMP(4);
    if (s_t.ipa_skip_filter) v.fskip |= bit(KSG_PL_INTER_POD_AFFINITY);
    const bool ipa_may_score = ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
                               !s_t.ipa_skip_score;
    const bool soft1 = g.pts_score && g.n_soft == 1;

    NodeEval ev[KN];
    int32_t fitr[KN], bar[KN];   // CAP: the raw NodeResourcesFit / BalancedAllocation scores
    int64_t yv[KN];
    int64_t pm[KN];   // one soft PTS constraint: the node's count m ...
    int32_t pr[KN];   // ... and pts_soft1_m's case (0 m valid, 1 no key, 2 ignored)
    int32_t nfeas = 0, minidx = 0x7fffffff, lign = 0, has_val = 0, has_zero = 0;
    long long max_t = 0, max_a = 0;
    long long mmin = BIG, mmax = -BIG - 1, imin = BIG, imax = -BIG - 1;
    int32_t lpres[kMaxSoft] = {0, 0, 0, 0}, lseen[kMaxSoft] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < KN; k++) {
      const int n = node_of(k);
      ev[k].st = 1;
      yv[k] = 0;
      pm[k] = 0;
      pr[k] = 2;
      if (n >= N || !ok) continue;
      TopoCtx tn = tc;
      tn.has_rec = true;
      tn.rec = srk[k];
      NodeCols L;
      if (KN == 1) L = Lreg;
      else load_cols(c, st.requested, st.nonzero, st.pod_count, n, L);
      ev[k] = eval_node_rec(c, prof, v, L, n, tn, cmp);
      KSG_CSTAMP(11);
      if (ev[k].st != 0) continue;
      if constexpr (CAP == 1 || CAP == 2) {
        fitr[k] = (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) ? (int32_t)fit_score(prof, p, L) : 0;
        bar[k] = (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) ? (int32_t)ba_score(prof, p, L) : 0;
      }
      nfeas += 1;
      minidx = min(minidx, n);
      max_t = max(max_t, (long long)ev[k].rt);
      max_a = max(max_a, (long long)ev[k].ra);
      if (g.pts_score) {
        if (g.require_all && !has_all(c, g.soft, g.n_soft, 6, n)) {
          lign += 1;
        } else {
#pragma unroll
          for (int i = 0; i < kMaxSoft; i++) {
            if (i >= g.n_soft) break;
            if (g.soft[6 * i + 5]) continue;
            const Slot& sl = s_t.soft[i];
            uint32_t val = lab(c, sl.col, n);
            if (!val) val = 1;
            if (sl.unique) {
              if (val == 1) lseen[i] = 1;
              else lpres[i] += 1;
            } else {
              atomicOr((uint32_t*)&s_hist[sl.mark + (val >> 5)], 1u << (val & 31));
            }
          }
        }
        if (soft1) {
          int64_t m = 0;
          const int r = pts_soft1_m(c, v, tn, n, m);
          pm[k] = m;
          pr[k] = r;
          if (r == 0) { has_val = 1; mmin = min(mmin, (long long)m); mmax = max(mmax, (long long)m); }
          else if (r == 1) has_zero = 1;
        }
      }
      KSG_CSTAMP(12);
      if (ipa_may_score) {
        yv[k] = ipa_score_node(c, prof, tn, n);
        imin = min(imin, (long long)yv[k]);
        imax = max(imax, (long long)yv[k]);
      }
    }
    KSG_CSTAMP(5);
    const bool need_ign = g.pts_score && g.require_all;
    bfold_i(nfeas, OpAddI{}, 0);
    bfold_i(minidx, OpMinI{}, 1);
    bfold_i((int32_t)max_t, OpMaxI32{}, 6);   // raw taint <= 255, raw node affinity <= 65535
    bfold_i((int32_t)max_a, OpMaxI32{}, 7);
    if (need_ign) bfold_i(lign, OpAddI{}, 2);
    if (soft1) {
      bfold_i(has_val, OpOrI{}, 3);
      bfold_i(has_zero, OpOrI{}, 4);
      bfold_l(mmin, OpMinL{}, 2);
      bfold_l(mmax, OpMaxL{}, 3);
    }
    if (need_se) {
#pragma unroll
      for (int i = 0; i < kMaxSoft; i++) {
        if (i >= g.n_soft) break;
        bfold_i(lpres[i], OpAddI{}, 8 + i);
        bfold_i(lseen[i], OpOrI{}, 12 + i);
      }
    }
    if (ipa_may_score) {
      bfold_l(imin, OpMinL{}, 4);
      bfold_l(imax, OpMaxL{}, 5);
    }
    __syncthreads();
    if (tid == 0) {
      s_wmin = get_i(1, OpMinI{});
      gst(&mine->nfeas, get_i(0, OpAddI{}));
      gst(&mine->minidx, s_wmin);
      gst(&mine->max_t, get_i(6, OpMaxI32{}));
      gst(&mine->max_a, get_i(7, OpMaxI32{}));
      if (need_ign) gst(&mine->n_ignored, get_i(2, OpAddI{}));
      if (soft1) {
        gst(&mine->has_val, get_i(3, OpOrI{}));
        gst(&mine->has_zero, get_i(4, OpOrI{}));
        gst(&mine->mmin, get_l(2, OpMinL{}));
        gst(&mine->mmax, get_l(3, OpMaxL{}));
      }
      if (need_se)
        for (int i = 0; i < g.n_soft; i++) {
          gst(&mine->soft_present[i], get_i(8 + i, OpAddI{}));
          gst(&mine->soft_seen[i], get_i(12 + i, OpOrI{}));
        }
      if (ipa_may_score) {
        gst(&mine->imin, get_l(4, OpMinL{}));
        gst(&mine->imax, get_l(5, OpMaxL{}));
      }
    }
    if (g.pts_score && ok)   // domains seen among feasible nodes (non-unique soft slots)
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        for (int wd = tid; wd < (sl.V + 31) / 32; wd += BLOCK) {
          if (pmode) gst(&myhist[sl.mark + wd], s_hist[sl.mark + wd]);
          else if (s_hist[sl.mark + wd]) gor(&acc->hist[sl.mark + wd], s_hist[sl.mark + wd]);
        }
      }
    KSG_CSTAMP(6);
    if (!coop_barrier(rbar, a.timeout, G, target)) return;
    KSG_CSTAMP(7);
    // CAP 2: the rows final since phase 2 (the status words and the raw
    // scores of every plugin but PodTopologySpread, whose raw count needs
    // phase 3's weights), written as if the pod is scored, go to the host now:
    // their PCIe transfer overlaps phase 3.  3c writes the rest, and zeroes
    // these when the pod turns out unscored (< 2 feasible nodes).
    uint32_t early_err = 0;
    const bool early = CAP == 2;
    if constexpr (CAP == 2) {
      if (early) {
        const size_t NN = N;
        const int es = a.cap_es;
        for (int k = 0; k < KN; k++) {
          const int n = node_of(k);
          if (n >= N) break;
          hst<true>(a.cap_fs + (size_t)kq * NN + n, ok ? ev[k].st : (uint32_t)KSG_FS_NOT_EVALUATED);
          const bool feas = ok && ev[k].st == 0;
          for (int q = 0; q < a.cap_n_rows; q++) {
            const int pl = a.cap_rows[q];
            if (pl == KSG_PL_POD_TOPOLOGY_SPREAD) continue;
            int64_t raw = 0;
            if (feas && ((v.smask >> pl) & 1u)) {
              switch (pl) {
                case KSG_PL_NODE_RESOURCES_FIT: raw = fitr[k]; break;
                case KSG_PL_BALANCED_ALLOCATION: raw = bar[k]; break;
                case KSG_PL_IMAGE_LOCALITY: raw = (int64_t)((srk[k] >> 32) & 0xff); break;
                case KSG_PL_TAINT_TOLERATION: raw = ev[k].rt; break;
                case KSG_PL_NODE_AFFINITY: raw = ev[k].ra; break;
                case KSG_PL_INTER_POD_AFFINITY: if (ipa_may_score) raw = yv[k]; break;
                default: break;
              }
            }
            cyc_put_es<true>(a.cap_raw, ((size_t)kq * a.cap_n_rows + q) * NN + n, raw, es);
            const bool f = es == 8 || (es == 4 ? raw == (int64_t)(int32_t)raw : raw == (int64_t)(int16_t)raw);
            early_err |= f ? 0u : 2u;
          }
        }
      }
    }

    // ---- phase 3: fold phase 2; sizes, normalisation, argmax --------------------
    // every reader of the tables and template tables for this pod is past
    // barrier 2: workgroup 0 applies the previous pod's assume to them now (the
    // next pod reads after barrier 3)
    if (wg == 0) lag_apply(cg, st, tt, s_lag, s_tables_ok != 0, s_lag_tab != 0);
    // the soft constraints' domain marks of every workgroup, loaded beside the
    // partial scalars below (one memory round trip for both; unused when the
    // pod turns out to have < 2 feasible nodes)
    if (g.pts_score && ok)
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        const int bw = (sl.V + 31) / 32;
        if (pmode) {   // or-ed into this workgroup's own marks
          fold_words(sl.mark, bw, true);
        } else {
          for (int wd = tid; wd < bw; wd += BLOCK) s_hist[sl.mark + wd] = gld(&acc->hist[sl.mark + wd]);
        }
      }
    {
      int32_t f_n = 0, f_min = 0x7fffffff, f_ign = 0, f_hv = 0, f_hz = 0, f_mt = 0, f_ma = 0;
      int32_t f_pr[kMaxSoft] = {0, 0, 0, 0}, f_se[kMaxSoft] = {0, 0, 0, 0};
      long long f_mmin = BIG, f_mmax = -BIG - 1, f_imin = BIG, f_imax = -BIG - 1;
      if (tid < G) {
        const CoopPart* q = parts + tid;
        f_n = gld(&q->nfeas);
        f_min = gld(&q->minidx);
        f_mt = (int32_t)gld(&q->max_t);
        f_ma = (int32_t)gld(&q->max_a);
        if (need_ign) f_ign = gld(&q->n_ignored);
        if (soft1) {
          f_hv = gld(&q->has_val);
          f_hz = gld(&q->has_zero);
          f_mmin = gld(&q->mmin);
          f_mmax = gld(&q->mmax);
        }
        if (need_se)
#pragma unroll
          for (int i = 0; i < kMaxSoft; i++)
            if (i < g.n_soft) { f_pr[i] = gld(&q->soft_present[i]); f_se[i] = gld(&q->soft_seen[i]); }
        if (ipa_may_score) {
          f_imin = gld(&q->imin);
          f_imax = gld(&q->imax);
        }
      }
      bfold_i(f_n, OpAddI{}, 0);
      bfold_i(f_min, OpMinI{}, 1);
      bfold_i(f_mt, OpMaxI32{}, 6);
      bfold_i(f_ma, OpMaxI32{}, 7);
      if (need_ign) bfold_i(f_ign, OpAddI{}, 2);
      if (soft1) {
        bfold_i(f_hv, OpOrI{}, 3);
        bfold_i(f_hz, OpOrI{}, 4);
        bfold_l(f_mmin, OpMinL{}, 2);
        bfold_l(f_mmax, OpMaxL{}, 3);
      }
      if (need_se) {
#pragma unroll
        for (int i = 0; i < kMaxSoft; i++) {
          if (i >= g.n_soft) break;
          bfold_i(f_pr[i], OpAddI{}, 8 + i);
          bfold_i(f_se[i], OpOrI{}, 12 + i);
        }
      }
      if (ipa_may_score) {
        bfold_l(f_imin, OpMinL{}, 4);
        bfold_l(f_imax, OpMaxL{}, 5);
      }
    }
    __syncthreads();
    KSG_CSTAMP(13);
    const int gnfeas = get_i(0, OpAddI{});
    const int gminidx = get_i(1, OpMinI{});
    const bool scored = ok && gnfeas >= 2;
    const bool do_pts = scored && g.pts_score;
    const bool do_ipa = scored && ipa_may_score;
    const int64_t gmax_t = get_i(6, OpMaxI32{}), gmax_a = get_i(7, OpMaxI32{});
    const long long gimin = do_ipa ? get_l(4, OpMinL{}) : 0, gimax = do_ipa ? get_l(5, OpMaxL{}) : 0;
    long long pmin = BIG, pmax = 0;
    if (do_pts) {   // (the marks were folded at the start of phase 3; the fold's barrier ordered them)
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        int bits = 0;
        for (int wd = tid; wd < (sl.V + 31) / 32; wd += BLOCK) bits += __popc((uint32_t)s_hist[sl.mark + wd]);
        bits = wave_sum32(bits);
        if (lane == 0 && bits) atomicAdd(&s_size[i], bits);
      }
      __syncthreads();
      if (tid == 0) {
        const int n_ign = need_ign ? get_i(2, OpAddI{}) : 0;
        for (int i = 0; i < g.n_soft; i++) {
          const Slot& sl = s_t.soft[i];
          int sz;
          if (g.soft[6 * i + 5]) sz = gnfeas - n_ign;
          else if (sl.unique) sz = get_i(8 + i, OpAddI{}) + get_i(12 + i, OpOrI{});
          else sz = s_size[i];
          s_t.soft_w[i] = sz + 2 < kCoopLog ? s_log[sz + 2] : c.log_table[sz + 2];   // math.Log(size + 2)
        }
      }
      __syncthreads();
      if (soft1) {
        long long lo = BIG, hi = 0;
        if (get_i(3, OpOrI{})) {
          lo = pts_soft1_score(g, s_t, get_l(2, OpMinL{}));
          hi = pts_soft1_score(g, s_t, get_l(3, OpMaxL{}));
        }
        if (get_i(4, OpOrI{})) { lo = min(lo, 0ll); hi = max(hi, 0ll); }
        pmin = lo;
        pmax = hi;
      } else {   // >= 2 soft constraints: raw scores first, then their extremes
        long long lo = BIG, hi = -BIG - 1;
#pragma unroll
        for (int k = 0; k < KN; k++) {
          const int n = node_of(k);
          if (n >= N || ev[k].st != 0) continue;
          TopoCtx tn = tc;
          tn.has_rec = true;
          tn.rec = srk[k];
          const int64_t x = pts_score_node(c, v, tn, n);
          if (x >= 0) { lo = min(lo, (long long)x); hi = max(hi, (long long)x); }
        }
        bfold_l(lo, OpMinL{}, 6);
        bfold_l(hi, OpMaxL{}, 7);
        __syncthreads();
        if (tid == 0) {
          gst(&mine->pmin, get_l(6, OpMinL{}));
          gst(&mine->pmax, get_l(7, OpMaxL{}));
        }
        if (!coop_barrier(rbar, a.timeout, G, target)) return;
        long long l2 = BIG, h2 = -BIG - 1;
        if (tid < G) {
          l2 = gld(&parts[tid].pmin);
          h2 = gld(&parts[tid].pmax);
        }
        bfold_l(l2, OpMinL{}, 8);
        bfold_l(h2, OpMaxL{}, 9);
        __syncthreads();
        l2 = get_l(8, OpMinL{});
        h2 = get_l(9, OpMaxL{});
        pmin = l2;
        pmax = l2 <= h2 ? h2 : 0;
      }
    }
    KSG_CSTAMP(14);
    uint64_t best = 0;
    uint32_t err = 0;
    // CAP: per node the weighted total, the normalised TaintToleration /
    // NodeAffinity / PodTopologySpread / InterPodAffinity scores and the raw
    // PodTopologySpread (negative: ignored node, recorded 0)
    int64_t ctot[KN], cnt_[KN], cna[KN], cps[KN], cis[KN], cpr[KN];
#pragma unroll
    for (int k = 0; k < KN; k++) ctot[k] = cnt_[k] = cna[k] = cps[k] = cis[k] = cpr[k] = 0;
    if (scored) {
      const int64_t w_pts = prof.weight[KSG_PL_POD_TOPOLOGY_SPREAD], w_ipa = prof.weight[KSG_PL_INTER_POD_AFFINITY];
#pragma unroll
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N || ev[k].st != 0) continue;
        int64_t total = total_score(v, ev[k].part, ev[k].rt, ev[k].ra, gmax_t, gmax_a, err,
                                    CAP ? &cnt_[k] : nullptr, CAP ? &cna[k] : nullptr);
        if (do_pts) {   // PodTopologySpread.NormalizeScore
          int64_t x;
          if (soft1) {   // from the count kept since sweep A: no loads
            x = pr[k] == 2 ? -1 : (pr[k] == 1 ? 0 : pts_soft1_score(g, s_t, pm[k]));
          } else {
            TopoCtx tn = tc;
            tn.has_rec = true;
            tn.rec = srk[k];
            x = pts_score_node(c, v, tn, n);
          }
          int64_t s;
          if (x < 0) s = 0;
          else if (pmax == 0) s = 100;
          else s = div_small(100 * (pmax + pmin - x), pmax);
          err |= (s < 0 || s > 100);
          total += s * w_pts;
          if constexpr (CAP != 0) { cps[k] = s; cpr[k] = x < 0 ? 0 : x; }
        }
        if (do_ipa) {   // InterPodAffinity.NormalizeScore (float64 min-max)
          const int64_t y = yv[k];
          const int64_t diff = gimax - gimin;
          double f = 0;
          if (diff > 0) f = (double)100 * ((double)(y - gimin) / (double)diff);
          const int64_t s = (int64_t)f;
          err |= (s < 0 || s > 100);
          total += s * w_ipa;
          if constexpr (CAP != 0) cis[k] = s;
        }
        const uint64_t key = argmax_key(total, n);
        best = key > best ? key : best;
        if constexpr (CAP != 0) ctot[k] = total;
      }
    }
    if constexpr (CAP == 1 || CAP == 2) {   // every row of this lane's nodes (ksg_capture semantics: < 2 feasible nodes record no scores)
      constexpr bool SYS = CAP == 2;
      const size_t NN = N;
      const int es = CAP == 2 ? a.cap_es : (a.cap_narrow ? 4 : 8);
      auto fits = [&](int64_t x) { return es == 8 || (es == 4 ? x == (int64_t)(int32_t)x : x == (int64_t)(int16_t)x); };
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N) break;
        const bool feas = scored && ev[k].st == 0;
        if (!early) hst<SYS>(a.cap_fs + (size_t)kq * NN + n, ok ? ev[k].st : (uint32_t)KSG_FS_NOT_EVALUATED);
        for (int q = 0; q < a.cap_n_rows; q++) {
          const int pl = a.cap_rows[q];
          // (written after barrier 2 with the same value when the pod is scored)
          const bool raw_done = early && scored && pl != KSG_PL_POD_TOPOLOGY_SPREAD;
          int64_t raw = 0, nrm = 0;
          if (feas && ((v.smask >> pl) & 1u)) {
            switch (pl) {
              case KSG_PL_NODE_RESOURCES_FIT: raw = fitr[k]; nrm = raw; break;
              case KSG_PL_BALANCED_ALLOCATION: raw = bar[k]; nrm = raw; break;
              case KSG_PL_IMAGE_LOCALITY: raw = (int64_t)((srk[k] >> 32) & 0xff); nrm = raw; break;
              case KSG_PL_TAINT_TOLERATION: raw = ev[k].rt; nrm = cnt_[k]; break;
              case KSG_PL_NODE_AFFINITY: raw = ev[k].ra; nrm = cna[k]; break;
              case KSG_PL_POD_TOPOLOGY_SPREAD: if (do_pts) { raw = cpr[k]; nrm = cps[k]; } break;
              case KSG_PL_INTER_POD_AFFINITY: if (do_ipa) { raw = yv[k]; nrm = cis[k]; } break;
              default: break;
            }
          }
          const size_t row = ((size_t)kq * a.cap_n_rows + q) * NN + n;
          if (!raw_done) {
            cyc_put_es<SYS>(a.cap_raw, row, raw, es);
            err |= fits(raw) ? 0u : 2u;
          }
          if (q < a.cap_n_normrows) {
            cyc_put_es<SYS>(a.cap_norm, ((size_t)kq * a.cap_n_normrows + q) * NN + n, nrm, es);
            err |= fits(nrm) ? 0u : 2u;
          }
        }
        const int64_t tv = feas ? ctot[k] : 0;
        cyc_put_es<SYS>(a.cap_tot, (size_t)kq * NN + n, tv, es);
        err |= fits(tv) ? 0u : 2u;
      }
    }
    err |= early_err;
    best = wreduce(best, OpMaxU64{});
    err = wreduce(err, OpOr32{});
    __syncthreads();   // every wave is past its get_*() reads of s_l / s_i
    if (lane == 0) { s_l[wv][10] = (long long)best; s_i[wv][13] = (int32_t)err; }
    __syncthreads();
    if (tid == 0) {
      unsigned long long b = 0;
      int32_t e = 0;
      for (int i = 0; i < NW; i++) { b = max(b, (unsigned long long)s_l[i][10]); e |= s_i[i][13]; }
      gst(&mine->best, b);
      gst(&mine->err, e);
      s_wbest = b;
      if constexpr (CAP == 3)
        if (e) __hip_atomic_fetch_or((__attribute__((address_space(1))) uint32_t*)&a.win_pod[row].err, (uint32_t)e,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (CAP == 3) {
      // A window row ends here, before any select or assume: every node's
      // static total, i.e. the weighted total less its NodeResourcesFit /
      // BalancedAllocation part, the only part an earlier pod of the window
      // can change (or -1: filtered out; 0: feasible, pod not scored); this
      // tile's kq + 1 best keys (the walk's best unchanged node is among them
      // when at most kq nodes changed); the pod's facts.  Agent-scope stores:
      // the walk reads them in this launch, from another workgroup.
      __shared__ WalkLds s_walk;
      __shared__ int s_final;
      const int n0 = node_of(0);
      const bool feas0 = ok && n0 < N && ev[0].st == 0;
      if (n0 < N)
        gst(a.win_tot + (size_t)row * N + n0, feas0 ? (scored ? (int32_t)(ctot[0] - (ev[0].part - ev[0].img)) : 0) : -1);
      uint64_t key = scored && feas0 ? argmax_key(ctot[0], n0) : 0;
      KSG_CSTAMP(8);
      for (int r = 0; r <= row; r++) {
        const uint64_t m = wreduce(key, OpMaxU64{});
        if (lane == 0) s_wtop[wv] = m;
        __syncthreads();
        uint64_t b = s_wtop[0];
        for (int i = 1; i < NW; i++) b = max(b, s_wtop[i]);
        if (tid == 0) gst(a.win_top + ((size_t)row * G + wg) * a.win_kmax + r, (unsigned long long)b);
        if (key == b) key = 0;
        __syncthreads();
      }
      if (wg == 0 && tid == 0) {
        WinPod* w = a.win_pod + row;
        uint32_t status = 0, score_skip = p.score_skip;
        if (ipa_in_filter && s_t.ipa_skip_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
        if (scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) && s_t.ipa_skip_score) {
          status |= KSG_ST_IPA_PRESCORE_SKIP;
          score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
        }
        bool fit_in = false;
        for (int kf = 0; kf < prof.n_filter; kf++) fit_in |= prof.filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
        gst(&w->ok, ok ? 1 : 0);
        gst(&w->nfeas, ok ? gnfeas : 0);
        gst(&w->minidx, gminidx);
        gst(&w->scored, scored ? 1 : 0);
        gst(&w->status, status);
        gst(&w->score_skip, score_skip);
        gst(&w->smask, v.smask);
        gst(&w->w_fit, v.w_fit);
        gst(&w->w_ba, v.w_ba);
        gst(&w->fit_on, fit_in && !((v.fskip >> KSG_PL_NODE_RESOURCES_FIT) & 1u) ? 1 : 0);
      }
      // this row's atomics set (soft marks; pre-pass histograms), read by
      // every workgroup of the row in phase 3: the last to arrive zeroes it
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)(a.arrive + row * 32),
                                                    1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (old + 1) % (unsigned)G == 0 ? 1 : 0;
      }
      __syncthreads();
      if (s_last)
        for (int i = tid; i < prev_fallback_words; i += BLOCK) gst(&acc->hist[i], 0);
      KSG_CSTAMP(9);
      // the last workgroup of each row (its row's outputs are performed: every
      // workgroup drained its stores before arriving) arrives on the launch's
      // counter, and the last row's walks the window.  (Every workgroup on
      // one counter: 185 atomics on one word serialise, ~5 us.)
      if (tid == 0) {
        int fin = 0;
        if (s_last) {
          const unsigned old = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)a.win_done, 1u,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          fin = old + 1 == (unsigned)count ? 1 : 0;
        }
        s_final = fin;
      }
      __syncthreads();
      if (s_final) {
        WalkArgs w;
        w.c = cg;
        w.st = st;
        w.tt = tt;
        w.use_tables = a.use_tables;
        w.cursor = const_cast<int32_t*>(a.win_cursor);
        w.win_base = a.win_base;
        w.G = G;
        w.K = a.win_kmax;
        w.win_tot = a.win_tot;
        w.win_top = a.win_top;
        w.win_pod = a.win_pod;
        w.prog = a.prog;
        w.placements = a.placements;
        w.results = a.results;
        w.wstats = a.win_stats;
        walk_window(w, first, count, prof, s_pods, s_walk);
        if (tid == 0) gst(a.win_done, 0u);
      }
      KSG_CSTAMP(10);
      continue;
    }
    if (CAP == 2) {
      // The per-cycle evaluation (one pod, no assume): no barrier 3.  Each
      // workgroup's host rows and argmax slot are performed (system-scope
      // stores: vmcnt(0)), it arrives on a counter, and the last of the G
      // arrivals selects the host and stores the result and then the flag
      // (ksg_eval_cycle's completion), so the rows' PCIe drain no longer
      // waits in a grid barrier before a phase 4 and the other workgroups end.
      KSG_CSTAMP(8);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)a.arrive, 1u,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (old + 1) % (unsigned)G == 0 ? 1 : 0;
      }
      __syncthreads();
      KSG_CSTAMP(9);
      if (s_last) {
        // the atomics set of this pod, read by every workgroup before its
        // arrival: clean for the next launch
        for (int i = tid; i < prev_fallback_words; i += BLOCK) gst(&acc->hist[i], 0);
        if (tid < 64) {
          unsigned long long b = 0;
          int32_t e = 0;
          for (int l = tid; l < G; l += 64) {
            b = max(b, (unsigned long long)gld(&parts[l].best));
            e |= gld(&parts[l].err);
          }
          b = wreduce(b, OpMaxU64{});
          e = wreduce(e, OpOrI{});
          if (tid == 0) {
            int selected = -1;
            uint32_t status = 0;
            if (!ok) {
              status |= KSG_ST_SCORE_ERROR;
            } else if (gnfeas == 1) {
              selected = gminidx;
            } else if (scored) {
              status |= KSG_ST_SCORED;
              if (e & 1) status |= KSG_ST_SCORE_ERROR;   // (bit 1: a capture value wider than the rows)
              else selected = key_node(b);
            }
            uint32_t score_skip = p.score_skip;
            if (ipa_in_filter && s_t.ipa_skip_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
            if (scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) && s_t.ipa_skip_score) {
              status |= KSG_ST_IPA_PRESCORE_SKIP;
              score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
            }
            a.placements[a.out0 + kq] = selected;
            ksg_result res;
            res.selected = selected;
            res.n_feasible = ok ? gnfeas : 0;
            res.status = status;
            res.score_skip = score_skip;
            if (a.results) a.results[a.out0 + kq] = res;
            hst<true>(a.h_ovf, (unsigned)((e >> 1) & 1));
            hst<true>(&a.h_res->selected, res.selected);
            hst<true>(&a.h_res->n_feasible, res.n_feasible);
            hst<true>(&a.h_res->status, res.status);
            hst<true>(&a.h_res->score_skip, res.score_skip);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.h_flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
      }
      KSG_CSTAMP(10);
      continue;   // (one pod)
    }
    if (a.commit && s_nlsel > 0) {   // the counts the assume will change (the winner's become the lag's)
      __syncthreads();
      const int nl = min(s_nlsel, kLagSel);
      const int bn = s_wbest ? key_node(s_wbest) : -1, mn = s_wmin;
#pragma unroll
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N) break;
        if (n == bn)
          for (int i = 0; i < nl; i++) gst(&mine->best_cnt[i], cnt_at(st.cnt, N, s_lsel[i], n));
        if (n == mn)
          for (int i = 0; i < nl; i++) gst(&mine->min_cnt[i], cnt_at(st.cnt, N, s_lsel[i], n));
      }
    }
    // the next pod's program words, loaded while this pod's last barrier waits
    nb_len = kq + 1 < count ? s_pods[kq + 1].blob_len : 0;
    if (nb_len <= kCoopPrefetch * BLOCK) {
      const int boff = kq + 1 < count ? s_pods[kq + 1].blob : 0;
#pragma unroll
      for (int u = 0; u < kCoopPrefetch; u++)
        nb[u] = tid + u * BLOCK < nb_len ? a.prog[boff + tid + u * BLOCK] : 0;
    }
    KSG_CSTAMP(8);
    if (!coop_barrier(rbar, a.timeout, G, target)) return;
    KSG_CSTAMP(9);

    // ---- phase 4: select and assume --------------------------------------------
    {
      unsigned long long b = 0;
      int32_t e = 0;
      if (tid < G) {
        b = gld(&parts[tid].best);
        e = gld(&parts[tid].err);
      }
      b = wreduce(b, OpMaxU64{});
      e = wreduce(e, OpOrI{});
      if (lane == 0) { s_l[wv][11] = (long long)b; s_i[wv][14] = e; }
    }
    __syncthreads();
    int selected = -1;
    uint32_t status = 0;
    if (!ok) {
      status |= KSG_ST_SCORE_ERROR;
    } else if (gnfeas == 1) {
      selected = gminidx;
    } else if (scored) {
      status |= KSG_ST_SCORED;
      unsigned long long b = 0;
      int32_t e = 0;
      for (int i = 0; i < NW; i++) { b = max(b, (unsigned long long)s_l[i][11]); e |= s_i[i][14]; }
      if (e & 1) status |= KSG_ST_SCORE_ERROR;   // (bit 1: a capture value wider than the rows, CAP == 2)
      else selected = key_node(b);
    }
    // the template tables reach tab one pod late unless the pod owns more
    // templates than the lag buffer holds
    const int32_t* cprog = p.commit >= 0 ? s_blob + (p.commit - p.blob) : nullptr;
    const int n_own_tmpl = cprog ? cprog[1 + cprog[0]] : 0;
    const bool tab_now = n_own_tmpl > kLagTmpl;
    if (a.commit && selected >= 0 && ((selected / BLOCK) % G) == wg && (selected % BLOCK) == tid)
    {
      coop_commit(cg, st, p, cprog, selected, tab_now);
      if (KN == 1) {   // the register copy
#pragma unroll
        for (int r = 0; r < KSG_MAX_RES; r++)
          if (r < cg.R) Lreg.req[r] += p.req[r];
        Lreg.nz_cpu += p.nz_cpu;
        Lreg.nz_mem += p.nz_mem;
        Lreg.pod_count += 1;
      }
    }
    __syncthreads();   // every wave is past this pod's reads of s_lag (applied by workgroup 0 in phase 3)
    {   // this pod's assume becomes the pending lag, in every workgroup alike
        // (lanes 0 .. n_sel - 1: the selectors' old counts; wave 1: the templates)
      LagDelta& d = s_lag;
      const int node = a.commit && selected >= 0 ? selected : -1;
      const bool any = node >= 0 && cprog;
      const int n_sel = any ? min(s_nlsel, kLagSel) : 0;
      const int n_tm = any && !tab_now ? n_own_tmpl : 0;
      if (tid < n_sel) {
        const int owner = (selected / BLOCK) % G;
        const int32_t* cnts = scored ? parts[owner].best_cnt : parts[owner].min_cnt;
        d.sel[tid] = s_lsel[tid];
        d.old_cnt[tid] = gld(cnts + tid);
      }
      if (tid >= 64 && tid < 64 + n_tm) {
        const int i = tid - 64;
        const int32_t* w = cprog + 2 + cprog[0];
        const int t = w[2 * i];
        const uint32_t val = cg.label_val[(size_t)cg.tmpl_col[t] * N + selected];
        d.tidx[i] = val ? cg.tmpl_off[t] + (int)val : -1;
        d.tw[i] = cg.tmpl_kind[t] == KSG_TMPL_PREF ? w[2 * i + 1] : 1;
        d.tt[i] = t;
      }
      if (tid == 0) {
        d.node = node;
        d.n_sel = n_sel;
        d.n_tmpl = n_tm;
        s_lag_tab = n_tm > 0 || (any && !tab_now) ? 1 : 0;
        s_prev_imm = any && tab_now ? 1 : 0;   // written at once by the owner lane: the next pod runs barrier 1
        if (any && s_nlsel > kLagSel) {   // more matched selectors than the lag holds: the tables go unused
          s_tables_ok = 0;
          if (wg == 0) gst(tt.invalid, 1u);
        }
      }
    }
    if (wg == 0 && kq == count - 1)   // the last pod's atomics set, read by everyone before barrier 3:
      for (int i = tid; i < prev_fallback_words; i += BLOCK) gst(&acc->hist[i], 0);   // clean for the next launch
    if (wg == 0 && tid == 0) {
      uint32_t score_skip = p.score_skip;
      if (ipa_in_filter && s_t.ipa_skip_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
      if (scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) && s_t.ipa_skip_score) {
        status |= KSG_ST_IPA_PRESCORE_SKIP;
        score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
      }
      a.placements[a.out0 + kq] = selected;
      ksg_result res;
      res.selected = selected;
      res.n_feasible = ok ? gnfeas : 0;
      res.status = status;
      res.score_skip = score_skip;
      if (a.results) a.results[a.out0 + kq] = res;
      if constexpr (CAP == 2) {   // every workgroup's host rows are done (barrier 3 drained them)
        int32_t ovf = 0;
        for (int i = 0; i < NW; i++) ovf |= s_i[i][14];
        hst<true>(a.h_ovf, (unsigned)((ovf >> 1) & 1));
        hst<true>(&a.h_res->selected, res.selected);
        hst<true>(&a.h_res->n_feasible, res.n_feasible);
        hst<true>(&a.h_res->status, res.status);
        hst<true>(&a.h_res->score_skip, res.score_skip);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.h_flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    KSG_CSTAMP(10);
  }
  // the last pod's assume: no reader follows in this launch
  __syncthreads();
  if (wg == 0) lag_apply(cg, st, tt, s_lag, s_tables_ok != 0, s_lag_tab != 0);
#ifdef KSG_STAMPS
  if (tid == 0 && wg == 0 && a.stamps)
    for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], st_acc[i]);
#endif
}
