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
};

__device__ __forceinline__ PodView make_view(const DevCluster& c, const ksg_profile& prof, const ksg_pod& p,
                                             const int32_t* P, const int32_t* gprog) {
  PodView v;
  const int boff = p.blob;
  auto rb = [boff](int off) { return off < 0 ? -1 : off - boff; };
  v.p = &p;
  v.P = P;
  v.na_req = rb(p.na_req);
  v.na_pref = rb(p.na_pref);
  v.img = rb(p.img);
  v.commit = rb(p.commit);
  v.tolf = P + rb(p.tol);
  v.tolp = v.tolf + c.W;
  v.node_set = p.node_set >= 0 ? gprog + p.node_set : nullptr;
  v.reject = (p.flags & KSG_POD_PREFILTER_REJECT) != 0;
  // PodTopologySpread / InterPodAffinity reach this evaluator only for pods
  // without terms (host check), i.e. they Skip.
  v.fskip = p.filter_skip | bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD);
  v.smask = prof.score_mask & ~p.score_skip & ~(bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD));
  v.w_fit = prof.weight[KSG_PL_NODE_RESOURCES_FIT];
  v.w_ba = prof.weight[KSG_PL_BALANCED_ALLOCATION];
  v.w_img = prof.weight[KSG_PL_IMAGE_LOCALITY];
  v.w_t = prof.weight[KSG_PL_TAINT_TOLERATION];
  v.w_a = prof.weight[KSG_PL_NODE_AFFINITY];
  return v;
}

struct NodeEval {
  uint32_t st;    // filter status word (0 = feasible)
  int64_t part;   // Σ weight x score over Fit, BalancedAllocation, ImageLocality
  int64_t rt;     // TaintToleration raw score
  int64_t ra;     // NodeAffinity raw score
};

// RunFilterPlugins (first rejection ends the node) + the raw Score() of every
// enabled score plugin, for one (pod, node).  craw/cnorm: optional capture rows.
__device__ __forceinline__ NodeEval eval_node(const DevCluster& c, const ksg_profile& prof, const PodView& v,
                                              const int64_t* requested, const int64_t* nonzero,
                                              const int32_t* pod_count, int n, int64_t* craw, int64_t* cnorm) {
  const ksg_pod& p = *v.p;
  const int N = c.N;
  NodeEval e{0, 0, 0, 0};
  uint32_t st = 0;
  if (v.reject || (v.node_set && !((((uint32_t)v.node_set[n >> 5]) >> (n & 31)) & 1u))) {
    st = KSG_FS_NOT_EVALUATED;
  } else {
    for (int kf = 0; kf < prof.n_filter && !st; kf++) {
      const int pl = prof.filter_order[kf];
      if ((v.fskip >> pl) & 1u) continue;
      switch (pl) {
        case KSG_PL_NODE_UNSCHEDULABLE:
          if (c.unsched[n] && !(p.flags & KSG_POD_TOL_UNSCHED)) st = pl + 1;
          break;
        case KSG_PL_NODE_NAME:
          if (p.node_name != -1 && p.node_name != n) st = pl + 1;
          break;
        case KSG_PL_TAINT_TOLERATION: {
          const int s = untolerated_slot(c, v.tolf, n);
          if (s >= 0) st = (uint32_t)(pl + 1) | ((uint32_t)s << 8);
          break;
        }
        case KSG_PL_NODE_AFFINITY:
          if (!na_required_match(c, v.P, v.na_req, n)) st = (uint32_t)(pl + 1) | (1u << 8);
          break;
        case KSG_PL_NODE_RESOURCES_FIT: {
          const uint32_t b = fit_filter(c, p, requested, pod_count[n], prof.fit_ignored_res, n);
          if (b) st = (uint32_t)(pl + 1) | (b << 8);
          break;
        }
        default:
          break;
      }
    }
  }
  e.st = st;
  if (st != 0) return e;
  if (v.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) {
    const int64_t s = fit_score(c, prof, p, requested, nonzero, n);
    e.part += s * v.w_fit;
    if (craw) { craw[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; cnorm[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; }
  }
  if (v.smask & bit(KSG_PL_BALANCED_ALLOCATION)) {
    const int64_t s = ba_score(c, prof, p, requested, nonzero, n);
    e.part += s * v.w_ba;
    if (craw) { craw[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; cnorm[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; }
  }
  if (v.smask & bit(KSG_PL_IMAGE_LOCALITY)) {
    const int64_t s = image_score(c, v.P, v.img, p.n_containers, n);
    e.part += s * v.w_img;
    if (craw) { craw[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; cnorm[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; }
  }
  if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) {
    e.rt = taint_score(c, v.tolp, n);
    if (craw) craw[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = e.rt;
  }
  if (v.smask & bit(KSG_PL_NODE_AFFINITY)) {
    e.ra = na_pref_score(c, v.P, v.na_pref, n);
    if (craw) craw[(size_t)KSG_PL_NODE_AFFINITY * N + n] = e.ra;
  }
  return e;
}

// DefaultNormalizeScore (reverse for TaintToleration) + weighted sum.  err set
// when a normalised score leaves [0, 100] (RunScorePlugins range check).
__device__ __forceinline__ int64_t total_score(const PodView& v, int64_t part, int64_t rt, int64_t ra, int64_t max_t,
                                               int64_t max_a, uint32_t& err, int64_t* nt, int64_t* na) {
  int64_t total = part;
  if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) {
    int64_t s = 100;
    if (max_t != 0) s = 100 - div_nonneg(100 * rt, max_t);
    err |= (s < 0 || s > 100);
    total += s * v.w_t;
    if (nt) *nt = s;
  }
  if (v.smask & bit(KSG_PL_NODE_AFFINITY)) {
    int64_t s = ra;
    if (max_a != 0) s = div_nonneg(100 * ra, max_a);
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
__device__ __forceinline__ void ipa_skip_bits(const ksg_profile& prof, const ksg_pod& p, uint32_t& status,
                                              uint32_t& score_skip) {
  score_skip = p.score_skip;
  if (p.ipa >= 0) return;
  bool ipa_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  if (ipa_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
  if ((status & KSG_ST_SCORED) && ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
      !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u)) {
    status |= KSG_ST_IPA_PRESCORE_SKIP;
    score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
  }
}

// NodeInfo.AddPod restricted to the columns the plugins read, plus the
// PodTopologySpread / InterPodAffinity count tables.
__device__ void commit_node(const DevCluster& c, int64_t* requested, int64_t* nonzero, int32_t* pod_count,
                            int32_t* cnt, int32_t* tab, int32_t* tmpl_total, const ksg_pod& p,
                            const int32_t* commit_prog, int n) {
  const int N = c.N;
  for (int r = 0; r < c.R; r++) requested[(size_t)r * N + n] += p.req[r];
  nonzero[n] += p.nz_cpu;
  nonzero[(size_t)N + n] += p.nz_mem;
  pod_count[n] += 1;
  if (commit_prog) {
    const int32_t* w = commit_prog;
    const int ns = *w++;
    for (int i = 0; i < ns; i++) cnt[(size_t)w[i] * N + n] += 1;
    w += ns;
    const int nt = *w++;
    for (int i = 0; i < nt; i++) {
      const int t = w[i];
      const int col = c.tmpl_col[t];
      const uint32_t val = c.label_val[(size_t)col * N + n];
      if (!val) continue;
      tab[c.tmpl_off[t] + val] += c.tmpl_kind[t] == KSG_TMPL_PREF ? c.tmpl_weight[t] : 1;
      tmpl_total[t] += 1;
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
