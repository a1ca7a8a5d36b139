// Kernels of libksched.so (gfx950).  See ksched.hip for the host side and
// DESIGN.md §3 for the structure.
#pragma once

#include "ksched_device.h"

namespace ksg {

constexpr uint32_t bit(int p) { return 1u << p; }

// ---- wave / block reductions (wave64: 6 xor-shuffle steps) ----------------
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ int32_t wave_sum32(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int32_t wave_min32(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

// ---- DPP wave reductions, result uniform (in SGPRs) ------------------------
// Quad swaps, half-row and row mirrors reduce each 16-lane row in four DPP
// moves; the four row values are combined through v_readlane.  No LDS
// traffic (a __shfl_xor step is a ds_bpermute round trip).  Call with all 64
// lanes active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
template <class T, class Op>
__device__ __forceinline__ T wreduce(T v, Op op) {
  if constexpr (sizeof(T) == 8) {
    v = op(v, (T)dpp64<0xB1>((uint64_t)v));    // quad_perm [1,0,3,2]
    v = op(v, (T)dpp64<0x4E>((uint64_t)v));    // quad_perm [2,3,0,1]
    v = op(v, (T)dpp64<0x141>((uint64_t)v));   // row_half_mirror
    v = op(v, (T)dpp64<0x140>((uint64_t)v));   // row_mirror
    const T r0 = (T)readlane64((uint64_t)v, 0), r1 = (T)readlane64((uint64_t)v, 16);
    const T r2 = (T)readlane64((uint64_t)v, 32), r3 = (T)readlane64((uint64_t)v, 48);
    return op(op(r0, r1), op(r2, r3));
  } else {
    v = op(v, (T)dpp32<0xB1>((uint32_t)v));
    v = op(v, (T)dpp32<0x4E>((uint32_t)v));
    v = op(v, (T)dpp32<0x141>((uint32_t)v));
    v = op(v, (T)dpp32<0x140>((uint32_t)v));
    const T r0 = (T)__builtin_amdgcn_readlane((int)v, 0), r1 = (T)__builtin_amdgcn_readlane((int)v, 16);
    const T r2 = (T)__builtin_amdgcn_readlane((int)v, 32), r3 = (T)__builtin_amdgcn_readlane((int)v, 48);
    return op(op(r0, r1), op(r2, r3));
  }
}
struct OpMaxU64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; } };
struct OpMax64 { __device__ int64_t operator()(int64_t a, int64_t b) const { return a > b ? a : b; } };
struct OpAdd32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMin32 { __device__ int32_t operator()(int32_t a, int32_t b) const { return a < b ? a : b; } };
struct OpOr32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; } };

// Workgroup barrier for LDS-only handoffs: waits for this wave's LDS traffic
// (lgkmcnt) but not for its global loads, which __syncthreads would drain
// (vmcnt(0)); for walks that keep the next step's global loads in flight
// across the barrier and read no global memory another wave wrote.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-pod values every lane needs, derived once from the LDS copy of the pod.
struct PodView {
  const ksg_pod* p;
  const int32_t* P;          // pod blob in LDS (offsets rebased to it)
  int na_req, na_pref, img, commit;
  const int32_t* tolf;       // toleration bitmap (all tolerations)
  const int32_t* tolp;       // toleration bitmap (PreferNoSchedule subset)
  const int32_t* node_set;   // PreFilterResult bitmap in global memory, or null
  bool reject;
  uint32_t fskip;            // filter plugins not run (PreFilter Skip)
  uint32_t smask;            // score plugins run (enabled and not PreScore Skip)
  int64_t w_fit, w_ba, w_img, w_t, w_a;
  int ports;                 // NodePorts program (blob-relative), -1 = none
  int vol;                   // volume plugins' program (blob-relative), -1 = none
  const uint32_t* used_ports;   // the replica's UsedPorts bitmaps (set by kernels that evaluate NodePorts)
};

// topo = false: PodTopologySpread / InterPodAffinity reach this evaluator only
// for pods without terms (host check), i.e. they Skip.  topo = true: the
// topology kernel evaluates them (IPA Skip decided on the device).
__device__ __forceinline__ PodView make_view(const DevCluster& c, const ksg_profile& prof, const ksg_pod& p,
                                             const int32_t* P, const int32_t* gprog, bool topo = false,
                                             const uint32_t* used_ports = nullptr) {
  PodView v;
  const int boff = p.blob;
  auto rb = [boff](int off) { return off < 0 ? -1 : off - boff; };
  v.p = &p;
  v.P = P;
  v.na_req = rb(p.na_req);
  v.na_pref = rb(p.na_pref);
  v.img = rb(p.img);
  v.commit = rb(p.commit);
  v.ports = rb(p.ports);
  v.vol = rb(p.vol);
  v.used_ports = used_ports;
  v.tolf = P + rb(p.tol);
  v.tolp = v.tolf + c.W;
  v.node_set = p.node_set >= 0 ? gprog + p.node_set : nullptr;
  v.reject = (p.flags & KSG_POD_PREFILTER_REJECT) != 0;
  if (topo) {
    v.fskip = p.filter_skip;
    v.smask = prof.score_mask & ~p.score_skip;
  } else {
    v.fskip = p.filter_skip | bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD);
    v.smask = prof.score_mask & ~p.score_skip & ~(bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD));
  }
  v.w_fit = prof.weight[KSG_PL_NODE_RESOURCES_FIT];
  v.w_ba = prof.weight[KSG_PL_BALANCED_ALLOCATION];
  v.w_img = prof.weight[KSG_PL_IMAGE_LOCALITY];
  v.w_t = prof.weight[KSG_PL_TAINT_TOLERATION];
  v.w_a = prof.weight[KSG_PL_NODE_AFFINITY];
  return v;
}

// ============================================================================
// PodTopologySpread / InterPodAffinity.
//
// The upstream plugins rescan every pod on every node in each PreFilter /
// PreScore [upstream podtopologyspread/filtering.go calPreFilterState,
// scoring.go PreScore; interpodaffinity/filtering.go PreFilter, scoring.go
// PreScore].  Here the scan is replaced by state maintained at assume time
// (commit_node):
//   cnt[s][n]      pods on node n matching selector s (namespace-scoped; one
//                  selector id per distinct PTS selector, IPA term selector and
//                  conjunction of a pod's required affinity terms)
//   tab[t][v]      per-domain table of term template t owned by existing pods
//                  (required anti-affinity / required affinity counts,
//                  preferred (anti-)affinity weight sums)
//   tmpl_total[t]  pods that contributed to template t
// and, per pod, a pre-pass over nodes folds cnt[s][.] into per-domain counts:
// directly per node when the topology column is unique (hostname), otherwise
// through LDS histograms indexed by the column's value id.
// ============================================================================
constexpr int kMaxHard = 4, kMaxSoft = 4, kMaxAff = 4, kMaxAnti = 4, kMaxPref = 8;

// A pointer into LDS.  Every parse_topo caller passes its LDS copy of the
// pod's programs, so the program pointers of TopoProg carry the LDS address
// space: a generic pointer read back from LDS would compile every program
// lookup on the per-node paths to a flat load (vmcnt + lgkmcnt wait each).
// (The host pass only sees the struct's declaration: a plain pointer there.)
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(3))) int32_t* lds_i32p;
#else
typedef const int32_t* lds_i32p;
#endif

struct TopoProg {
  int n_hard, n_soft, require_all;
  lds_i32p hard;   // {col sel max_skew min_domains self_match na nt} x n_hard
  lds_i32p soft;   // {col sel max_skew na nt is_hostname} x n_soft
  int n_aff, sel_all, self_all;
  lds_i32p aff_cols;
  int n_anti;
  lds_i32p anti;   // {col sel}
  int n_pref;
  lds_i32p pref;   // {col sel weight}
  int n_ma, n_mh, n_mp;
  lds_i32p m_anti, m_hard, m_pref;
  bool pts_filter, pts_score, ipa;
};

// One LDS histogram slot: counts (V words) + presence bitmap + optional mark bitmap.
struct Slot {
  int col, sel, unique, V, hist, pres, mark;
};

struct TopoShared {
  Slot hard[kMaxHard], soft[kMaxSoft], aff[kMaxAff], anti[kMaxAnti], pref[kMaxPref];
  long long hard_min[kMaxHard];
  int hard_dom[kMaxHard];
  long long soft_empty[kMaxSoft];     // unique soft column: count of the "" domain
  int soft_present[kMaxSoft];         // unique soft column: feasible non-ignored nodes with a value
  int soft_empty_seen[kMaxSoft];
  double soft_w[kMaxSoft];
  int n_ignored;
  long long aff_total;
  int pref_any;
  int ipa_skip_filter;                // InterPodAffinity PreFilter Skip
  int ipa_skip_score;                 // InterPodAffinity PreScore Skip
  int words;
  int ok;
};

// Static record of a (pod, node) (ksg_sweep_static): bits 0-4 filter verdicts
// (1 = rejects), 8-15 raw TaintToleration, 16-31 raw NodeAffinity, 32-39 raw
// ImageLocality, 40-55 the node's first untolerated NoSchedule / NoExecute
// taint slot (TaintToleration's status payload).
constexpr uint32_t kSrUnsched = 1u, kSrNodeName = 2u, kSrTaint = 4u, kSrNodeAff = 8u, kSrNotEval = 16u;
constexpr int kSrTaintSlotShift = 40;

struct TopoCtx {
  const TopoProg* g;
  const TopoShared* s;
  const int32_t* hist;   // LDS
  const int32_t* cnt;    // replica's cnt[S][N]
  const int32_t* tab;    // replica's template tables
  bool coherent;         // tab is written by other workgroups of this launch (ksg_topo_coop):
                         // read it with agent-scope atomic loads, never from a cache line
  bool has_rec;          // rec = the node's static record: inclusion() reads its verdict bits
  uint64_t rec;
  // ksg_topo_coop: the previous pod's assume reaches tab one pod late; these
  // entries (index, added weight) are added by the reader meanwhile
  const int32_t* lag_idx = nullptr;
  const int32_t* lag_w = nullptr;
  int lag_n = 0;
  __device__ __forceinline__ int32_t tabv(int idx) const {
    int32_t v;
    if (coherent)   // agent-scope global (sc1) load: no stale L1 line, no acquire needed
      v = __hip_atomic_load((__attribute__((address_space(1))) int32_t*)(const_cast<int32_t*>(tab) + idx),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      v = tab[idx];
    for (int i = 0; i < lag_n; i++) v += lag_idx[i] == idx ? lag_w[i] : 0;
    return v;
  }
};

__device__ __forceinline__ void parse_topo(const ksg_pod& p, const int32_t* P, uint32_t fskip, uint32_t smask,
                                           TopoProg& g) {
  g = TopoProg{};
  const int boff = p.blob;
  if (p.pts >= 0) {
    lds_i32p w = (lds_i32p)(P + (p.pts - boff));
    g.n_hard = w[0];
    g.n_soft = w[1];
    g.require_all = w[2];
    g.hard = w + 3;
    g.soft = g.hard + 7 * g.n_hard;
  }
  g.pts_filter = g.n_hard > 0 && !((fskip >> KSG_PL_POD_TOPOLOGY_SPREAD) & 1u);
  g.pts_score = g.n_soft > 0 && ((smask >> KSG_PL_POD_TOPOLOGY_SPREAD) & 1u);
  if (p.ipa >= 0) {
    lds_i32p w = (lds_i32p)(P + (p.ipa - boff));
    g.n_aff = w[0];
    g.sel_all = w[1];
    g.self_all = w[2];
    g.aff_cols = w + 3;
    w += 3 + g.n_aff;
    g.n_anti = *w++;
    g.anti = w;
    w += 2 * g.n_anti;
    g.n_pref = *w++;
    g.pref = w;
    w += 3 * g.n_pref;
    g.n_ma = *w++;
    g.m_anti = w;
    w += g.n_ma;
    g.n_mh = *w++;
    g.m_hard = w;
    w += g.n_mh;
    g.n_mp = *w++;
    g.m_pref = w;
    g.ipa = true;
  }
}

// One thread: lay out this pod's LDS histograms.
__device__ __forceinline__ void layout_slots(const DevCluster& c, const TopoProg& g, TopoShared& s) {
  int words = 0;
  const bool ok = g.n_hard <= kMaxHard && g.n_soft <= kMaxSoft && g.n_aff <= kMaxAff && g.n_anti <= kMaxAnti &&
                  g.n_pref <= kMaxPref;
  auto mk = [&](Slot& sl, int col, int sel, bool need_mark) {
    sl.col = col;
    sl.sel = sel;
    sl.unique = c.col_unique[col];
    sl.V = c.col_vocab[col];
    sl.hist = sl.pres = sl.mark = -1;
    if (!sl.unique) {
      sl.hist = words;
      words += sl.V;
      sl.pres = words;
      words += (sl.V + 31) / 32;
      if (need_mark) {
        sl.mark = words;
        words += (sl.V + 31) / 32;
      }
    }
  };
  if (ok) {
    for (int i = 0; i < g.n_hard; i++) mk(s.hard[i], g.hard[7 * i], g.hard[7 * i + 1], false);
    for (int i = 0; i < g.n_soft; i++) mk(s.soft[i], g.soft[6 * i], g.soft[6 * i + 1], true);
    for (int i = 0; i < g.n_aff; i++) mk(s.aff[i], g.aff_cols[i], g.sel_all, false);
    for (int i = 0; i < g.n_anti; i++) mk(s.anti[i], g.anti[2 * i], g.anti[2 * i + 1], false);
    for (int i = 0; i < g.n_pref; i++) mk(s.pref[i], g.pref[3 * i], g.pref[3 * i + 1], false);
  }
  s.words = words;
  s.ok = ok && words <= KSG_HIST_MAX;
}

__device__ __forceinline__ int32_t cnt_at(const int32_t* cnt, int N, int sel, int n) {
  return sel < 0 ? 0 : cnt[(size_t)sel * N + n];
}
__device__ __forceinline__ uint32_t lab(const DevCluster& c, int col, int n) {
  return c.label_val[(size_t)col * c.lab_stride + (n - c.lab_base)];
}
__device__ __forceinline__ bool has_all(const DevCluster& c, const int32_t* cons, int ncons, int stride, int n) {
  for (int i = 0; i < ncons; i++)
    if (!lab(c, cons[stride * i], n)) return false;
  return true;
}
// topologySpreadConstraint.matchNodeInclusionPolicies
__device__ __forceinline__ bool inclusion(const DevCluster& c, const PodView& v, int na, int nt, int n) {
  const GNode nd{&c, n};
  if (na && !na_required_match(nd, v.P, v.na_req)) return false;
  if (nt && untolerated_slot(c, nd, v.tolf) >= 0) return false;
  return true;
}
// the same from the node's static record when the context carries one (the
// record's NodeAffinity / TaintToleration bits are these two evaluations)
__device__ __forceinline__ bool inclusion(const DevCluster& c, const PodView& v, const TopoCtx& t, int na, int nt,
                                          int n) {
  if (t.has_rec) return !(na && (t.rec & kSrNodeAff)) && !(nt && (t.rec & kSrTaint));
  return inclusion(c, v, na, nt, n);
}
__device__ __forceinline__ bool bit_get(const int32_t* h, int base, uint32_t v) {
  return ((((uint32_t)h[base + (v >> 5)]) >> (v & 31)) & 1u) != 0;
}
// count in the domain of node n for a non-unique slot (0 when the domain is absent)
__device__ __forceinline__ int64_t hist_at(const int32_t* h, const Slot& sl, uint32_t v) {
  return bit_get(h, sl.pres, v) ? (int64_t)h[sl.hist + v] : 0;
}

// PodTopologySpread.Filter: 0 pass, 1 missing required label, 2 skew.
__device__ __forceinline__ uint32_t pts_filter_node(const DevCluster& c, const PodView& v, const TopoCtx& t, int n) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  const bool all = has_all(c, g.hard, g.n_hard, 7, n);
  for (int i = 0; i < g.n_hard; i++) {
    const int32_t* h = g.hard + 7 * i;
    const uint32_t val = lab(c, h[0], n);
    if (!val) return 1;
    const Slot& sl = s.hard[i];
    int64_t m;
    if (sl.unique) m = (all && inclusion(c, v, t, h[5], h[6], n)) ? cnt_at(t.cnt, c.N, sl.sel, n) : 0;
    else m = hist_at(t.hist, sl, val);
    if (m + h[4] - s.hard_min[i] > h[2]) return 2;
  }
  return 0;
}

// InterPodAffinity.Filter: 0 pass, 1 affinity, 2 anti-affinity, 3 existing pods' anti-affinity.
__device__ __forceinline__ uint32_t ipa_filter_node(const DevCluster& c, const TopoCtx& t, int n) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  bool pods_exist = true;
  for (int i = 0; i < g.n_aff; i++) {
    const Slot& sl = s.aff[i];
    const uint32_t val = lab(c, sl.col, n);
    if (!val) return 1;
    const int64_t m = sl.unique ? cnt_at(t.cnt, c.N, g.sel_all, n) : hist_at(t.hist, sl, val);
    if (m <= 0) pods_exist = false;
  }
  if (!pods_exist && !(s.aff_total == 0 && g.n_aff > 0 && g.self_all)) return 1;
  for (int i = 0; i < g.n_anti; i++) {
    const Slot& sl = s.anti[i];
    const uint32_t val = lab(c, sl.col, n);
    if (!val) continue;
    const int64_t m = sl.unique ? cnt_at(t.cnt, c.N, sl.sel, n) : hist_at(t.hist, sl, val);
    if (m > 0) return 2;
  }
  for (int i = 0; i < g.n_ma; i++) {
    const int tm = g.m_anti[i];
    const uint32_t val = lab(c, c.tmpl_col[tm], n);
    if (val && t.tabv(c.tmpl_off[tm] + val) > 0) return 3;
  }
  return 0;
}

// PodTopologySpread.Score; -1 for IgnoredNodes.
__device__ __forceinline__ int64_t pts_score_node(const DevCluster& c, const PodView& v, const TopoCtx& t, int n) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  if (g.require_all && !has_all(c, g.soft, g.n_soft, 6, n)) return -1;
  double score = 0.0;
  for (int i = 0; i < g.n_soft; i++) {
    const int32_t* sc = g.soft + 6 * i;
    const uint32_t val = lab(c, sc[0], n);
    if (!val) continue;
    const Slot& sl = s.soft[i];
    int64_t m;
    if (sc[5]) m = cnt_at(t.cnt, c.N, sl.sel, n);                    // hostname: this node's pods
    else if (!sl.unique) m = t.hist[sl.hist + val];
    else if (val == 1) m = s.soft_empty[i];
    else m = inclusion(c, v, t, sc[3], sc[4], n) ? cnt_at(t.cnt, c.N, sl.sel, n) : 0;
    const double x = (double)m * s.soft_w[i];
    score += x + (double)(sc[2] - 1);
  }
  return (int64_t)round(score);
}

// InterPodAffinity.Score
__device__ __forceinline__ int64_t ipa_score_node(const DevCluster& c, const ksg_profile& prof, const TopoCtx& t,
                                                  int n) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  int64_t sc = 0;
  for (int i = 0; i < g.n_pref; i++) {
    const Slot& sl = s.pref[i];
    const uint32_t val = lab(c, sl.col, n);
    if (!val) continue;
    const int64_t m = sl.unique ? cnt_at(t.cnt, c.N, sl.sel, n) : hist_at(t.hist, sl, val);
    sc += (int64_t)g.pref[3 * i + 2] * m;
  }
  if (prof.hard_pod_affinity_weight > 0)
    for (int i = 0; i < g.n_mh; i++) {
      const int tm = g.m_hard[i];
      const uint32_t val = lab(c, c.tmpl_col[tm], n);
      if (val) sc += (int64_t)prof.hard_pod_affinity_weight * t.tabv(c.tmpl_off[tm] + val);
    }
  for (int i = 0; i < g.n_mp; i++) {
    const int tm = g.m_pref[i];
    const uint32_t val = lab(c, c.tmpl_col[tm], n);
    if (val) sc += t.tabv(c.tmpl_off[tm] + val);
  }
  return sc;
}

struct NodeEval {
  uint32_t st;    // filter status word (0 = feasible)
  int64_t part;   // Σ weight x score over Fit, BalancedAllocation, ImageLocality
  int64_t rt;     // TaintToleration raw score
  int64_t ra;     // NodeAffinity raw score
  int64_t img;    // weight x ImageLocality score (part of `part`)
};

// RunFilterPlugins (first rejection ends the node) + the raw Score() of every
// enabled score plugin, for one (pod, node).  craw/cnorm: optional capture rows;
// lraw: optional per-plugin raw scores of the node-local plugins ([KSG_NPLUGINS],
// constant indices: registers).
// Src: GNode (columns in global memory) or LNode (a node cached in LDS); L:
// the node's resource columns, already gathered by the caller.
#ifdef KSG_STAMPS
// Diagnostic build only: per-segment cycles of eval_node_src, lane 0 of
// workgroup 0 (slot 0 the node-set check, 1 + p filter plugin p, 13 the Fit /
// BalancedAllocation scores, 14 ImageLocality + TaintToleration, 15 NodeAffinity).
#ifdef KSG_PART
static   // a part's own copy (diagnostic stamps are read from the host TU's)
#endif
__device__ unsigned long long g_eval_stamp[16];
#define KSG_ESTAMP(k)                                                          \
  do {                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                         \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                \
    if (threadIdx.x == 0 && blockIdx.x == 0) { g_eval_stamp[k] += _t - _es_last; } \
    _es_last = _t;                                                             \
    __builtin_amdgcn_sched_barrier(0);                                         \
  } while (0)
#else
#define KSG_ESTAMP(k) do {} while (0)
#endif

// cm: the profile's CmProf when the caller computed it (Fit + BalancedAllocation
// then take fit_ba_cm when cm->fast).
template <class Src>
__device__ __forceinline__ NodeEval eval_node_src(const DevCluster& c, const ksg_profile& prof, const PodView& v,
                                                  const Src& nd, const NodeCols& L, int n, int64_t* craw,
                                                  int64_t* cnorm, const TopoCtx* tc = nullptr,
                                                  int64_t* lraw = nullptr, const CmProf* cm = nullptr) {
  const ksg_pod& p = *v.p;
  const int N = c.N;
  NodeEval e{0, 0, 0, 0, 0};
  uint32_t st = 0;
#ifdef KSG_STAMPS
  unsigned long long _es_last = __builtin_amdgcn_s_memtime();
#endif
  if (v.reject || (v.node_set && !((((uint32_t)v.node_set[n >> 5]) >> (n & 31)) & 1u))) {
    st = KSG_FS_NOT_EVALUATED;
  } else {
    KSG_ESTAMP(0);
    for (int kf = 0; kf < prof.n_filter && !st; kf++) {
      const int pl = prof.filter_order[kf];
      if ((v.fskip >> pl) & 1u) continue;
#ifdef KSG_STAMPS
      struct EStampOnExit {   // the plugin's slot, stamped when its case ends
        unsigned long long& last;
        int k;
        __device__ ~EStampOnExit() {
          __builtin_amdgcn_sched_barrier(0);
          const unsigned long long t = __builtin_amdgcn_s_memtime();
          if (threadIdx.x == 0 && blockIdx.x == 0) g_eval_stamp[k] += t - last;
          last = t;
          __builtin_amdgcn_sched_barrier(0);
        }
      } _es_guard{_es_last, 1 + (pl < 12 ? pl : 11)};
#endif
      switch (pl) {
        case KSG_PL_NODE_UNSCHEDULABLE:
          if (nd.unsched() && !(p.flags & KSG_POD_TOL_UNSCHED)) st = pl + 1;
          break;
        case KSG_PL_NODE_NAME:
          if (p.node_name != -1 && p.node_name != n) st = pl + 1;
          break;
        case KSG_PL_TAINT_TOLERATION: {
          const int s = untolerated_slot(c, nd, v.tolf);
          if (s >= 0) st = (uint32_t)(pl + 1) | ((uint32_t)s << 8);
          break;
        }
        case KSG_PL_NODE_AFFINITY:
          if (!na_required_match(nd, v.P, v.na_req)) st = (uint32_t)(pl + 1) | (1u << 8);
          break;
        case KSG_PL_NODE_PORTS:   // reached only by pods with host ports (PreFilter Skip otherwise)
          if (v.ports >= 0 && v.used_ports && ports_conflict(v.used_ports, N, n, v.P + v.ports)) st = pl + 1;
          break;
        case KSG_PL_NODE_RESOURCES_FIT: {
          const uint32_t b = fit_filter(c, p, L, prof.fit_ignored_res);
          if (b) st = (uint32_t)(pl + 1) | (b << 8);
          break;
        }
        case KSG_PL_POD_TOPOLOGY_SPREAD:
          if (tc && tc->g->pts_filter) {
            const uint32_t r = pts_filter_node(c, v, *tc, n);
            if (r) st = (uint32_t)(pl + 1) | (r << 8);
          }
          break;
        case KSG_PL_INTER_POD_AFFINITY:
          if (tc && tc->g->ipa) {
            const uint32_t r = ipa_filter_node(c, *tc, n);
            if (r) st = (uint32_t)(pl + 1) | (r << 8);
          }
          break;
        // volume plugins: reached only by pods with claims (PreFilter Skip
        // otherwise); NodeVolumeLimits passes (no CSI attach limits modelled)
        case KSG_PL_VOLUME_RESTRICTIONS:
          if (v.vol >= 0 && (v.P[v.vol] & 1)) st = pl + 1;
          break;
        case KSG_PL_VOLUME_BINDING:
          if (v.vol >= 0) {
            const VolVerdict r = vol_filter(nd, v.P, v.vol, n);
            if (r.vb) st = (uint32_t)(pl + 1) | (r.vb << 8);
          }
          break;
        case KSG_PL_VOLUME_ZONE:
          if (v.vol >= 0 && vol_filter(nd, v.P, v.vol, n).vz) st = pl + 1;
          break;
        default:
          break;
      }
    }
  }
  e.st = st;
  if (st != 0) return e;
  KSG_ESTAMP(0);
  if (cm && cm->fast && (v.smask & (bit(KSG_PL_NODE_RESOURCES_FIT) | bit(KSG_PL_BALANCED_ALLOCATION)))) {
    int64_t sf, sb;
    fit_ba_cm(*cm, p, L, sf, sb);
    if (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) {
      e.part += sf * v.w_fit;
      if (lraw) lraw[KSG_PL_NODE_RESOURCES_FIT] = sf;
      if (craw) { craw[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = sf; cnorm[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = sf; }
    }
    if (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) {
      e.part += sb * v.w_ba;
      if (lraw) lraw[KSG_PL_BALANCED_ALLOCATION] = sb;
      if (craw) { craw[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = sb; cnorm[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = sb; }
    }
  } else {
  if (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) {
    const int64_t s = fit_score(prof, p, L);
    e.part += s * v.w_fit;
    if (lraw) lraw[KSG_PL_NODE_RESOURCES_FIT] = s;
    if (craw) { craw[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; cnorm[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; }
  }
  if (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) {
    const int64_t s = ba_score(prof, p, L);
    e.part += s * v.w_ba;
    if (lraw) lraw[KSG_PL_BALANCED_ALLOCATION] = s;
    if (craw) { craw[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; cnorm[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; }
  }
  }
  KSG_ESTAMP(13);
  if (v.smask & bit(KSG_PL_IMAGE_LOCALITY)) {
    const int64_t s = image_score(c, nd, v.P, v.img, p.n_containers);
    e.img = s * v.w_img;
    if (lraw) lraw[KSG_PL_IMAGE_LOCALITY] = s;
    e.part += e.img;
    if (craw) { craw[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; cnorm[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; }
  }
  if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) {
    e.rt = taint_score(c, nd, v.tolp);
    if (lraw) lraw[KSG_PL_TAINT_TOLERATION] = e.rt;
    if (craw) craw[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = e.rt;
  }
  KSG_ESTAMP(14);
  if (v.smask & bit(KSG_PL_NODE_AFFINITY)) {
    e.ra = na_pref_score(nd, v.P, v.na_pref);
    if (lraw) lraw[KSG_PL_NODE_AFFINITY] = e.ra;
    if (craw) craw[(size_t)KSG_PL_NODE_AFFINITY * N + n] = e.ra;
  }
  KSG_ESTAMP(15);
  return e;
}

__device__ __forceinline__ NodeEval eval_node(const DevCluster& c, const ksg_profile& prof, const PodView& v,
                                              const int64_t* requested, const int64_t* nonzero,
                                              const int32_t* pod_count, int n, int64_t* craw, int64_t* cnorm,
                                              const TopoCtx* tc = nullptr) {
  NodeCols L;
  load_cols(c, requested, nonzero, pod_count, n, L);
  return eval_node_src(c, prof, v, GNode{&c, n}, L, n, craw, cnorm, tc);
}

// DefaultNormalizeScore (reverse for TaintToleration) + weighted sum.  err set
// when a normalised score leaves [0, 100] (RunScorePlugins range check).
__device__ __forceinline__ int64_t total_score(const PodView& v, int64_t part, int64_t rt, int64_t ra, int64_t max_t,
                                               int64_t max_a, uint32_t& err, int64_t* nt, int64_t* na) {
  int64_t total = part;
  if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) {
    int64_t s = 100;
    if (max_t != 0) s = 100 - div_small(100 * rt, max_t);
    err |= (s < 0 || s > 100);
    total += s * v.w_t;
    if (nt) *nt = s;
  }
  if (v.smask & bit(KSG_PL_NODE_AFFINITY)) {
    int64_t s = ra;
    if (max_a != 0) s = div_small(100 * ra, max_a);
    err |= (s < 0 || s > 100);
    total += s * v.w_a;
    if (na) *na = s;
  }
  return total;
}

__device__ __forceinline__ uint64_t argmax_key(int64_t total, int n) {
  // selectHost with the deterministic tie-break: highest total, then lowest node index
  return ((uint64_t)total << 32) | (uint64_t)(0xffffffffu - (uint32_t)n);
}
__device__ __forceinline__ int key_node(uint64_t key) { return (int)(0xffffffffu - (uint32_t)(key & 0xffffffffu)); }

// InterPodAffinity without any term of, or matching, this pod: PreFilter and
// PreScore both return Skip [upstream interpodaffinity/filtering.go, scoring.go].
__device__ __forceinline__ bool ipa_in_filter(const ksg_profile& prof) {
  bool ipa_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  return ipa_filter;
}
// ipa_filter: ipa_in_filter(prof), hoisted out of per-pod loops by callers on a critical path
__device__ __forceinline__ void ipa_skip_bits(const ksg_profile& prof, bool ipa_filter, const ksg_pod& p,
                                              uint32_t& status, uint32_t& score_skip) {
  score_skip = p.score_skip;
  if (p.ipa >= 0) return;
  if (ipa_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
  if ((status & KSG_ST_SCORED) && ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
      !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u)) {
    status |= KSG_ST_IPA_PRESCORE_SKIP;
    score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
  }
}
__device__ __forceinline__ void ipa_skip_bits(const ksg_profile& prof, const ksg_pod& p, uint32_t& status,
                                              uint32_t& score_skip) {
  ipa_skip_bits(prof, ipa_in_filter(prof), p, status, score_skip);
}

// NodeInfo.AddPod restricted to the columns the plugins read, plus the
// PodTopologySpread / InterPodAffinity count tables.
// sign = +1: assume (NodeInfo.AddPod); sign = -1: a preemption victim's
// deletion (NodeInfo.RemovePod), the exact inverse.
__device__ void commit_node(const DevCluster& c, int64_t* requested, int64_t* nonzero, int32_t* pod_count,
                            int32_t* cnt, int32_t* tab, int32_t* tmpl_total, const ksg_pod& p,
                            const int32_t* commit_prog, int n, int sign = 1, uint32_t* ports = nullptr,
                            const int32_t* ports_prog = nullptr) {
  const int N = c.N;
  if (ports && ports_prog) ports_commit(ports, N, n, ports_prog, sign);
  for (int r = 0; r < c.R; r++) requested[(size_t)r * N + n] += sign * p.req[r];
  nonzero[n] += sign * p.nz_cpu;
  nonzero[(size_t)N + n] += sign * p.nz_mem;
  pod_count[n] += sign;
  if (commit_prog) {
    const int32_t* w = commit_prog;
    const int ns = *w++;
    for (int i = 0; i < ns; i++) cnt[(size_t)w[i] * N + n] += sign;
    w += ns;
    const int nt = *w++;
    for (int i = 0; i < nt; i++) {
      const int t = w[2 * i];
      const int col = c.tmpl_col[t];
      const uint32_t val = c.label_val[(size_t)col * N + n];
      if (!val) continue;
      tab[c.tmpl_off[t] + val] += sign * (c.tmpl_kind[t] == KSG_TMPL_PREF ? w[2 * i + 1] : 1);
      tmpl_total[t] += sign;
    }
  }
}

// Stage pod `pi` (record + program blob) into LDS.  Caller brackets with barriers.
template <int BLOCK>
__device__ __forceinline__ void stage_pod(const ksg_pod* pods, const int32_t* prog, int pi, ksg_pod* s_pod,
                                          int32_t* s_blob) {
  const int tid = threadIdx.x;
  if (tid < (int)(sizeof(ksg_pod) / 4))
    reinterpret_cast<int32_t*>(s_pod)[tid] = reinterpret_cast<const int32_t*>(pods + pi)[tid];
  const int boff = pods[pi].blob, blen = pods[pi].blob_len;
  for (int i = tid; i < blen; i += BLOCK) s_blob[i] = prog[boff + i];
}

}  // namespace ksg
