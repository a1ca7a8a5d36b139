// Device-side data layout and per-node plugin arithmetic for gfx950.
//
// One workgroup owns one scheduling replica.  The pod's programs (tolerations,
// node-affinity programs, images, topology terms) are staged into LDS once
// per pod and read by every lane; node columns are read coalesced (lane i of
// a wave touches node base+i of the same column).  Nothing in this path is a
// dense contraction, so MFMA is not used: the per-node work is int64 compares,
// int64 divides and a handful of float64 ops, bound by L2/HBM bytes and by the
// per-pod barrier latency.
//
// Arithmetic restated from the upstream plugins [upstream k8s.io/kubernetes
// v1.32 pkg/scheduler/framework/plugins/...], identical to oracle/oracle.cpp;
// compiled with -ffp-contract=off so float64 follows Go's (unfused) operation
// order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ksched.h"

#define KSG_BLOB_MAX 4096          // LDS words for one pod's programs
#define KSG_HIST_MAX 8192          // LDS words for per-pod domain histograms

struct DevCluster {
  int32_t N, R, L, T, I, V, W;     // W = toleration bitmap words
  const int64_t* alloc;            // [R][N]
  const int32_t* allowed;          // [N]
  const uint8_t* unsched;          // [N]
  const uint32_t* label_val;       // [L][N]
  const int64_t* label_num;        // [L][N]
  const uint8_t* label_num_ok;     // [L][N]
  const uint32_t* taints;          // [T][N]
  const uint8_t* taint_effect;     // [V]
  const uint32_t* images;          // [I][N]
  // per-node reciprocals of the cpu and memory allocatable (memory in MiB; 1
  // for a zero column), for the 32-bit Fit / BalancedAllocation forms:
  // v_rcp_f32 estimates for qdiv32 and ddiv_rcp for float64 ddiv_r
  const float2* rcp32;             // [N]
  const double2* rcp64;            // [N]
  // topology
  int32_t S, n_tmpl;
  const int32_t* tmpl_col;
  const int32_t* tmpl_kind;
  const int32_t* tmpl_weight;
  const int32_t* tmpl_off;         // [n_tmpl] offset of the template's domain table
  const int32_t* col_vocab;        // [L]
  const uint8_t* col_unique;       // [L]
  const double* log_table;
  int32_t log_n;
  int32_t PW;                      // NodePorts: words of a node's UsedPorts bitmap (host-port vocabulary / 32)
  // label_val addressing: value of (col, n) at label_val[col * lab_stride + n -
  // lab_base] (N / 0; ksg_topo_coop points a private copy at the lane nodes'
  // labels staged in LDS)
  int32_t lab_stride, lab_base;
};

// Mutable per-replica state.  Replica r's arrays start at base + r * stride.
struct DevState {
  int64_t* requested;   // [R][N]
  int64_t* nonzero;     // [2][N]
  int32_t* pod_count;   // [N]
  int32_t* cnt;         // [S][N]   pods on node n matching selector s
  int32_t* tab;         // [Σ template table sizes]  per-domain template tables
  int32_t* tmpl_total;  // [n_tmpl] pods that contributed to template t
  // scratch (per replica)
  int64_t* partial;     // [N] Σ weight × score of un-normalised plugins, -1 = infeasible
  int64_t* sraw;        // [4][N] raw scores of normalised plugins (taint, NA, PTS, IPA)
  uint32_t* ports;      // [PW][N]  NodeInfo.UsedPorts as a bitmap over the host-port vocabulary
  size_t stride_req, stride_nz, stride_pc, stride_cnt, stride_tab, stride_tt, stride_part, stride_sraw,
      stride_ports;
};

// nodeports.fitsPorts: does any id of the pod's conflict list sit in the
// node's UsedPorts?  (HostPortInfo.CheckConflict, resolved on the host into
// vocabulary ids: ksched.h ksg_pod.ports.)
__device__ __forceinline__ bool ports_conflict(const uint32_t* used, int N, int n, const int32_t* w) {
  const int nconf = w[0];
  bool hit = false;
  for (int i = 0; i < nconf; i++) {
    const uint32_t id = (uint32_t)w[1 + i];
    hit = hit || ((used[(size_t)(id >> 5) * N + n] >> (id & 31)) & 1u);
  }
  return hit;
}
// NodeInfo.updateUsedPorts: Add (sign > 0) / Remove (sign < 0) the pod's own
// ids.  A set, as HostPortInfo is: Remove drops the entry even if another pod
// on the node uses the same (IP, protocol, port).
__device__ __forceinline__ void ports_commit(uint32_t* used, int N, int n, const int32_t* w, int sign) {
  const int32_t* own = w + 1 + w[0];
  const int nown = own[0];
  for (int i = 0; i < nown; i++) {
    const uint32_t id = (uint32_t)own[1 + i];
    uint32_t& word = used[(size_t)(id >> 5) * N + n];
    if (sign > 0) word |= 1u << (id & 31);
    else word &= ~(1u << (id & 31));
  }
}

__device__ __forceinline__ int64_t ld64(const int32_t* w) {
  return (int64_t)(((uint64_t)(uint32_t)w[1] << 32) | (uint32_t)w[0]);
}

// Exact Go int64 division x / a for 0 <= x, 0 < a (every division on this
// path: dividends are scores x 100 or byte counts x 100, divisors are
// allocatable amounts or maxima).  gfx950 has no int64 divide instruction;
// the compiler's software divide is ~100 instructions.  Below 2^52 the f64
// quotient is within one of the truth, and one integer multiply-subtract
// corrects it, so the result is exact.
__device__ __forceinline__ int64_t div_nonneg(int64_t x, int64_t a) {
  if ((uint64_t)x >= (1ull << 52) || (uint64_t)(a - 1) >= (1ull << 52)) return x / a;
  int64_t q = (int64_t)((double)x / (double)a);
  int64_t r = x - q * a;
  if (r < 0) { q -= 1; r += a; }
  if (r >= a) { q += 1; }
  return q;
}

// floor(x / a) for 0 <= x, 0 < a, quotient below 2^20 (every division on the
// changed-node path: scores x 100 over allocatable amounts, weight sums or
// maxima).  inv = (float)(1 / a).  The f32 estimate is within 2^-21 relative
// of x / a, i.e. within one of the quotient; one integer multiply-subtract
// corrects it, so the result is exact.
__device__ __forceinline__ int64_t qdiv(int64_t x, int64_t a, float inv) {
  const float xf = __builtin_fmaf((float)(uint32_t)((uint64_t)x >> 32), 4294967296.0f, (float)(uint32_t)x);
  int64_t q = (int32_t)(xf * inv);
  const int64_t r = x - q * a;
  q += r < 0 ? -1 : (r >= a ? 1 : 0);
  return q;
}

// x / a in float64, bit-identical to the compiler's division for 0 <= x and
// 1 <= a < 2^53 (integers): the same rcp + two Newton steps + residual fma
// sequence without v_div_scale / v_div_fmas / v_div_fixup, which are identities
// in that range.  No VCC use, so two divisions interleave.
__device__ __forceinline__ double ddiv_rcp(double a) {   // ddiv's reciprocal of a
  double r = __builtin_amdgcn_rcp(a);
  double e = __builtin_fma(-a, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-a, r, 1.0);
  return __builtin_fma(r, e, r);
}
// ddiv with r = ddiv_rcp(a) computed once per divisor (same bits)
__device__ __forceinline__ double ddiv_r(double x, double a, double r) {
  const double q = x * r;
  const double rem = __builtin_fma(-a, q, x);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ double ddiv(double x, double a) { return ddiv_r(x, a, ddiv_rcp(a)); }

// qdiv in 32 bits: floor(x / a) for 0 <= x < 2^30, a >= 1 and a quotient of
// at most ~100 (the one-step correction covers the float estimate's error).
__device__ __forceinline__ int32_t qdiv32(int32_t x, int32_t a, float inv) {
  int32_t q = (int32_t)((float)x * inv);
  const int32_t r = x - q * a;
  q += r < 0 ? -1 : (r >= a ? 1 : 0);
  return q;
}

// floor(x / a) for a quotient known to be at most 100 (scores, normalisation):
// qdiv with its own reciprocal estimate; div_nonneg outside qdiv's domain.
__device__ __forceinline__ int64_t div_small(int64_t x, int64_t a) {
  if (x < 0 || a <= 0) return x / a;
  return qdiv(x, a, __builtin_amdgcn_rcpf((float)a));
}

// ---- node sources ------------------------------------------------------------
// The plugin code reads a node's static columns through an accessor (GNode:
// the SoA columns in global memory), so a kernel can substitute its own copy.
struct GNode {
  const DevCluster* c;
  int n;
  __device__ __forceinline__ uint32_t label(int col) const {
    return c->label_val[(size_t)col * c->lab_stride + (n - c->lab_base)];
  }
  __device__ __forceinline__ bool num(int col, int64_t& x) const {
    const size_t k = (size_t)col * c->N + n;
    if (!c->label_num_ok[k]) return false;
    x = c->label_num[k];
    return true;
  }
  __device__ __forceinline__ uint32_t taint(int s) const { return c->taints[(size_t)s * c->N + n]; }
  __device__ __forceinline__ uint8_t effect(uint32_t vid) const { return c->taint_effect[vid]; }
  __device__ __forceinline__ uint32_t image(int s) const { return c->images[(size_t)s * c->N + n]; }
  __device__ __forceinline__ bool unsched() const { return c->unsched[n] != 0; }
};

// ---- requirement programs (encoder.py grammar); P = pod blob in LDS -------
template <class Src>
__device__ __forceinline__ bool eval_req(const Src& nd, const int32_t*& w) {
  const int col = w[0], op = w[1], nv = w[2];
  const int32_t* vals = w + 3;
  w += 3 + nv;
  if (op == 6) return false;
  const uint32_t v = nd.label(col);
  if (op == 0 || op == 1) {
    bool hit = false;
    for (int i = 0; i < nv; i++) hit |= ((uint32_t)vals[i] == v);
    if (op == 0) return v != 0 && hit;
    return v == 0 || !hit;
  }
  if (op == 2) return v != 0;
  if (op == 3) return v == 0;
  if (v == 0) return false;
  int64_t x;
  if (!nd.num(col, x)) return false;
  const int64_t bound = ld64(vals);
  return op == 4 ? x > bound : x < bound;
}

template <class Src>
__device__ __forceinline__ bool eval_term(const Src& nd, const int32_t*& w) {
  const int nr = *w++;
  bool ok = nr > 0;
  for (int i = 0; i < nr; i++) ok = eval_req(nd, w) && ok;
  return ok;
}

template <class Src>
__device__ __forceinline__ bool na_required_match(const Src& nd, const int32_t* P, int na_req) {
  if (na_req < 0) return true;
  const int32_t* w = P + na_req;
  const int nsel = *w++;
  bool ok = true;
  for (int i = 0; i < nsel; i++) ok = eval_req(nd, w) && ok;
  if (!ok) return false;
  const int nterms = *w++;
  if (nterms < 0) return true;
  bool any = false;
  for (int t = 0; t < nterms; t++) any = eval_term(nd, w) || any;
  return any;
}

template <class Src>
__device__ __forceinline__ int64_t na_pref_score(const Src& nd, const int32_t* P, int na_pref) {
  const int32_t* w = P + na_pref;
  const int nterms = *w++;
  int64_t s = 0;
  for (int t = 0; t < nterms; t++) {
    const int weight = *w++;
    if (eval_term(nd, w)) s += weight;
  }
  return s;
}

// ---- volume plugins' Filter over the pod's volume program ----------------
// (encoder.py Encoder._volume_plan grammar; upstream v1.32
// volumerestrictions.Filter's ReadWriteOncePod check, volumebinding
// FindPodVolumes (checkBoundClaims, the selected-node fast path,
// checkVolumeProvisions), volumezone.Filter)
struct VolVerdict {
  bool rwop;          // VolumeRestrictions: a running pod holds a ReadWriteOncePod claim
  uint32_t vb;        // VolumeBinding reason bits: 1 node conflict, 2 bind conflict, 4 PV missing
  bool vz;            // VolumeZone: no available volume zone
};

template <class Src>
__device__ __forceinline__ bool any_term(const Src& nd, const int32_t*& w, int nt) {
  bool any = false;
  for (int t = 0; t < nt; t++) any = eval_term(nd, w) || any;
  return any;
}

template <class Src>
__device__ __forceinline__ VolVerdict vol_filter(const Src& nd, const int32_t* P, int vol, int n) {
  VolVerdict r{false, 0, false};
  const int32_t* w = P + vol;
  r.rwop = (*w++ & 1) != 0;
  // bound claims, in volume order: the first missing PV or affinity mismatch ends the check
  const int nb = *w++;
  bool done = false;
  for (int b = 0; b < nb; b++) {
    const int kind = *w++;
    if (kind == 0) {
      if (!done) r.vb |= 4u;
      done = true;
      continue;
    }
    const int nt = *w++;
    if (nt < 0) continue;
    const bool ok = any_term(nd, w, nt);
    if (!done && !ok) {
      r.vb |= 1u;
      done = true;
    }
  }
  // unbound WaitForFirstConsumer claims: selected node, then provisioning
  const int np = *w++;
  bool prov_ok = true;
  for (int k = 0; k < np; k++) {
    const int sel = *w++;
    const int nt = *w++;
    if (sel != -1 && sel != n) prov_ok = false;
    if (nt < 0) prov_ok = false;
    else if (nt > 0 && !any_term(nd, w, nt)) prov_ok = false;
  }
  if (!prov_ok) r.vb |= 2u;
  // VolumeZone: a node without any topology label passes
  bool constrained = false;
  for (int k = 0; k < 4; k++) {
    const int col = w[k];
    constrained = constrained || (col >= 0 && nd.label(col) != 0);
  }
  w += 4;
  const int nz = *w++;
  for (int k = 0; k < nz; k++) {
    const int col = w[0], gcol = w[1];
    const int nv = w[2];
    const int32_t* ids = w + 3;
    const int ng = w[3 + nv];
    const int32_t* gids = w + 4 + nv;
    w += 4 + nv + ng;
    uint32_t v = nd.label(col);
    const int32_t* set = ids;
    int ns = nv;
    if (!v) {   // the beta label missing: the GA one
      v = nd.label(gcol);
      set = gids;
      ns = ng;
    }
    bool hit = false;
    for (int i = 0; i < ns; i++) hit |= (uint32_t)set[i] == v;
    if (constrained && (!v || !hit)) r.vz = true;
  }
  return r;
}

__device__ __forceinline__ bool tol_bit(const int32_t* tolp, uint32_t vid) {
  return (((uint32_t)tolp[vid >> 5]) >> (vid & 31)) & 1u;
}

// FindMatchingUntoleratedTaint (NoSchedule | NoExecute): slot or -1.
template <class Src>
__device__ __forceinline__ int untolerated_slot(const DevCluster& c, const Src& nd, const int32_t* tolf) {
  for (int s = 0; s < c.T; s++) {
    const uint32_t id = nd.taint(s);
    if (!id) break;
    const uint32_t vid = id - 1;
    const uint8_t e = nd.effect(vid);
    if (e != KSG_EFFECT_NO_SCHEDULE && e != KSG_EFFECT_NO_EXECUTE) continue;
    if (!tol_bit(tolf, vid)) return s;
  }
  return -1;
}

template <class Src>
__device__ __forceinline__ int64_t taint_score(const DevCluster& c, const Src& nd, const int32_t* tolp) {
  int64_t k = 0;
  for (int s = 0; s < c.T; s++) {
    const uint32_t id = nd.taint(s);
    if (!id) break;
    const uint32_t vid = id - 1;
    if (nd.effect(vid) != KSG_EFFECT_PREFER_NO_SCHEDULE) continue;
    k += !tol_bit(tolp, vid);
  }
  return k;
}

// A node's resource columns, gathered with independent loads up front so
// their latencies overlap (the plugin code below branches on them).
struct NodeCols {
  int64_t alloc[KSG_MAX_RES];
  int64_t req[KSG_MAX_RES];     // NodeInfo.Requested
  int64_t nz_cpu, nz_mem;       // NodeInfo.NonZeroRequested
  int32_t pod_count, allowed;
};

__device__ __forceinline__ void load_cols(const DevCluster& c, const int64_t* requested, const int64_t* nonzero,
                                          const int32_t* pod_count, int n, NodeCols& L) {
  const size_t N = c.N;
#pragma unroll
  for (int r = 0; r < KSG_MAX_RES; r++) {
    L.alloc[r] = r < c.R ? c.alloc[r * N + n] : 0;
    L.req[r] = r < c.R ? requested[r * N + n] : 0;
  }
  L.nz_cpu = nonzero[n];
  L.nz_mem = nonzero[N + n];
  L.pod_count = pod_count[n];
  L.allowed = c.allowed[n];
}

// a[r] for a wave-uniform runtime r without dynamic register indexing (a
// uniform branch per column keeps a[] in VGPRs; an indexed access would put
// the whole array in scratch memory).
__device__ __forceinline__ int64_t pick(const int64_t (&a)[KSG_MAX_RES], int r) {
  switch (r) {
    case 0: return a[0];
    case 1: return a[1];
    case 2: return a[2];
    case 3: return a[3];
    case 4: return a[4];
    case 5: return a[5];
    case 6: return a[6];
    default: return a[7];
  }
}

// noderesources.fitsRequest: bit0 pods, bit(r+1) resource column r
__device__ __forceinline__ uint32_t fit_filter(const DevCluster& c, const ksg_pod& p, const NodeCols& L,
                                               uint32_t ignored) {
  uint32_t bits = 0;
  if ((int64_t)L.pod_count + 1 > (int64_t)L.allowed) bits |= 1u;
#pragma unroll
  for (int r = 0; r < KSG_MAX_RES; r++) {
    if (r >= c.R) break;
    const int64_t q = p.req[r];
    if (q <= 0) continue;
    if (r >= 3 && ((ignored >> r) & 1u)) continue;
    if (q > L.alloc[r] - L.req[r]) bits |= 1u << (r + 1);
  }
  return bits;
}

// resourceAllocationScorer.calculateResourceAllocatableRequest
__device__ __forceinline__ void alloc_req(const ksg_pod& p, const NodeCols& L, int r, bool use_requested,
                                          int64_t& a, int64_t& q) {
  int64_t pr;
  if (use_requested) pr = p.req[r];
  else pr = r == KSG_RES_CPU ? p.nz_cpu : (r == KSG_RES_MEM ? p.nz_mem : p.req[r]);
  a = 0;
  q = 0;
  if (pr == 0 && r >= 3) return;
  a = pick(L.alloc, r);
  int64_t base;
  if (!use_requested && r == KSG_RES_CPU) base = L.nz_cpu;
  else if (!use_requested && r == KSG_RES_MEM) base = L.nz_mem;
  else base = pick(L.req, r);
  q = base + pr;
}

// helper.BuildBrokenLinearFunction over the profile's shape (scores already
// x 10): the first point at or above p, interpolated from the one before
// [upstream v1.32 pkg/scheduler/framework/plugins/helper/shape_score.go]
__device__ __forceinline__ int64_t rtcr_shape(const ksg_profile& prof, int64_t p) {
  for (int i = 0; i < prof.shape_n; i++) {
    const int64_t u = prof.shape_util[i];
    if (p <= u) {
      if (i == 0) return prof.shape_score[0];
      const int64_t u0 = prof.shape_util[i - 1], s0 = prof.shape_score[i - 1];
      return s0 + (prof.shape_score[i] - s0) * (p - u0) / (u - u0);   // Go's truncating division
    }
  }
  return prof.shape_n > 0 ? prof.shape_score[prof.shape_n - 1] : 0;
}

// NodeResourcesFit's score: LeastAllocated / MostAllocated (integer means),
// RequestedToCapacityRatio (the shape at each resource's utilization, only
// positive scores weighted, the mean rounded half away from zero)
// [upstream v1.32 noderesources/least_allocated.go, most_allocated.go,
// requested_to_capacity_ratio.go]
__device__ __forceinline__ int64_t fit_score(const ksg_profile& prof, const ksg_pod& p, const NodeCols& L) {
  int64_t num = 0, wsum = 0;
  const bool rtcr = prof.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO;
  for (int i = 0; i < prof.fit_n; i++) {
    int64_t a, q;
    alloc_req(p, L, prof.fit_res[i], false, a, q);
    if (a == 0) continue;
    int64_t s;
    if (rtcr) {
      s = rtcr_shape(prof, q > a ? 100 : q * 100 / a);
      if (s <= 0) continue;
    } else if (prof.fit_strategy == KSG_LEAST_ALLOCATED) {
      s = q > a ? 0 : div_small((a - q) * 100, a);
    } else {
      s = div_small((q > a ? a : q) * 100, a);
    }
    num += s * prof.fit_w[i];
    wsum += prof.fit_w[i];
  }
  if (wsum == 0) return 0;
  if (rtcr) return (int64_t)round((double)num / (double)wsum);
  return div_small(num, wsum);
}

// balancedResourceScorer, in Go's float64 operation order.  Fractions are
// recomputed in the second pass instead of stored (no private-memory array).
__device__ __forceinline__ int64_t ba_score(const ksg_profile& prof, const ksg_pod& p, const NodeCols& L) {
  int k = 0;
  double total = 0.0, f0 = 0.0, f1 = 0.0;
  for (int i = 0; i < prof.ba_n; i++) {
    int64_t a, q;
    alloc_req(p, L, prof.ba_res[i], true, a, q);
    if (a == 0) continue;
    double f = ddiv((double)q, (double)a);   // IEEE-exact for integer q >= 0, a >= 1
    if (f > 1) f = 1;
    total += f;
    if (k == 0) f0 = f;
    else if (k == 1) f1 = f;
    k++;
  }
  double sd = 0.0;
  if (k == 2) {
    sd = fabs((f0 - f1) / 2);
  } else if (k > 2) {
    const double mean = total / (double)k;
    double sum = 0.0;
    for (int i = 0; i < prof.ba_n; i++) {
      int64_t a, q;
      alloc_req(p, L, prof.ba_res[i], true, a, q);
      if (a == 0) continue;
      double f = ddiv((double)q, (double)a);   // IEEE-exact for integer q >= 0, a >= 1
      if (f > 1) f = 1;
      sum = sum + (f - mean) * (f - mean);
    }
    sd = sqrt(sum / (double)k);
  }
  return (int64_t)((1 - sd) * (double)100);
}

// Batch-uniform profile facts for the compact evaluator.
struct CmProf {
  bool fast;        // Fit and BalancedAllocation both score exactly {cpu, memory}
  bool least;
  int64_t wc, wm;   // Fit resource weights of cpu / memory
  float inv_ws, inv_wc, inv_wm;   // 1 / (wc + wm), 1 / wc, 1 / wm
};

__device__ __forceinline__ CmProf cm_prof(const ksg_profile& prof) {
  CmProf m{false, prof.fit_strategy == KSG_LEAST_ALLOCATED, 0, 0, 1.0f, 1.0f, 1.0f};
  bool ok = prof.fit_n == 2 && prof.ba_n == 2 && prof.fit_strategy != KSG_REQUESTED_TO_CAPACITY_RATIO;
  if (ok) {
    const int r0 = prof.fit_res[0], r1 = prof.fit_res[1];
    ok = (r0 == KSG_RES_CPU && r1 == KSG_RES_MEM) || (r0 == KSG_RES_MEM && r1 == KSG_RES_CPU);
    m.wc = r0 == KSG_RES_CPU ? prof.fit_w[0] : prof.fit_w[1];
    m.wm = r0 == KSG_RES_CPU ? prof.fit_w[1] : prof.fit_w[0];
    const int b0 = prof.ba_res[0], b1 = prof.ba_res[1];
    ok = ok && ((b0 == KSG_RES_CPU && b1 == KSG_RES_MEM) || (b0 == KSG_RES_MEM && b1 == KSG_RES_CPU));
    ok = ok && m.wc > 0 && m.wm > 0;
  }
  m.fast = ok;
  if (ok) {
    m.inv_ws = 1.0f / (float)(m.wc + m.wm);
    m.inv_wc = 1.0f / (float)m.wc;
    m.inv_wm = 1.0f / (float)m.wm;
  }
  return m;
}

// fit_score + ba_score for a CmProf::fast profile (both over exactly {cpu,
// memory}): the same arithmetic without branches or loops over the profile's
// resource lists, so the two chains interleave (sweep_cm_scores' restatement
// on a node's gathered columns).  Equal to fit_score / ba_score bit for bit.
__device__ __forceinline__ void fit_ba_cm(const CmProf& m, const ksg_pod& p, const NodeCols& L, int64_t& fit,
                                          int64_t& ba) {
  const int64_t ac = L.alloc[KSG_RES_CPU], am = L.alloc[KSG_RES_MEM];
  const bool hc = ac > 0, hm = am > 0;
  const int64_t sac = hc ? ac : 1, sam = hm ? am : 1;
  const float ic = __builtin_amdgcn_rcpf((float)sac), im = __builtin_amdgcn_rcpf((float)sam);
  const int64_t qc = L.nz_cpu + p.nz_cpu, qm = L.nz_mem + p.nz_mem;
  int64_t xc, xm;
  if (m.least) {
    xc = qc > ac ? 0 : (ac - qc) * 100;
    xm = qm > am ? 0 : (am - qm) * 100;
  } else {
    xc = (qc > ac ? ac : qc) * 100;
    xm = (qm > am ? am : qm) * 100;
  }
  const int64_t sc = qdiv(xc, sac, ic), sm = qdiv(xm, sam, im);
  const int64_t num = (hc ? sc * m.wc : 0) + (hm ? sm * m.wm : 0);
  const int64_t ws = (hc ? m.wc : 0) + (hm ? m.wm : 0);
  fit = ws == 0 ? 0 : qdiv(num, ws, __builtin_amdgcn_rcpf((float)ws));
  double fc = ddiv((double)(L.req[KSG_RES_CPU] + p.req[KSG_RES_CPU]), (double)sac);
  double fm = ddiv((double)(L.req[KSG_RES_MEM] + p.req[KSG_RES_MEM]), (double)sam);
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = hc && hm ? fabs((fc - fm) / 2) : 0.0;
  ba = (int64_t)((1 - sd) * (double)100);
}

template <class Src>
__device__ __forceinline__ int64_t image_score(const DevCluster& c, const Src& nd, const int32_t* P, int img,
                                               int n_containers) {
  int64_t sum = 0;
  if (img >= 0) {
    const int32_t* w = P + img;
    const int cnt = *w++;
    for (int i = 0; i < cnt; i++, w += 3) {
      const uint32_t id = (uint32_t)w[0];
      const int64_t contrib = ld64(w + 1);
      for (int s = 0; s < c.I; s++) {
        const uint32_t x = nd.image(s);
        if (!x || x > id) break;
        if (x == id) { sum += contrib; break; }
      }
    }
  }
  const int64_t mb = 1024 * 1024, minT = 23 * mb;
  const int64_t mx = 1000 * mb * (int64_t)n_containers;
  if (sum < minT) sum = minT;
  else if (sum > mx) sum = mx;
  return div_small(100 * (sum - minT), mx - minT);
}
