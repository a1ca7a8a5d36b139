// The exact 32-bit NodeResourcesFit / BalancedAllocation evaluation of one
// pod on one live node row (the N32 forms: memory in MiB, every reachable sum
// below 2^30 / 2^31, per-node reciprocals with an exact correction), used by
// the speculate-and-verify walk's verification (ksched_phase2v.h) to evaluate
// each new row version for the batch's pods.  Included by ksched_dev.h inside
// namespace ksk after ksg_batch_phase2s (SlotLayout, CmProf, P1Stats).
// (Round 2's transposed walk, ksg_batch_phase2t, was built on these helpers;
// it was retired in round 6: never faster than the window slot walk, and the
// spec walk superseded both.)

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
