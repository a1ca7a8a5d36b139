// Replica sweep (configs 4/5: R what-if scheduler profiles over one queue on
// one cluster), included by ksched.hip inside its anonymous namespace.
//
// Of the per-(pod, node) work, everything except NodeResourcesFit and
// BalancedAllocation is independent of the replica: the NodeUnschedulable,
// NodeName, TaintToleration and NodeAffinity verdicts and the raw
// TaintToleration, NodeAffinity and ImageLocality scores depend on the pod and
// the node's static columns only (the profiles change which plugins run and
// their weights, not what a plugin computes).  So:
//
//   ksg_sweep_static   grid (node tiles, batch pods): one 8-byte static record
//                      per (pod, node), computed once for all replicas;
//   ksg_sweep<BLOCK,KN> S workgroups per replica, persistent over the batch:
//                      per pod, one sweep over the replica's nodes reads the
//                      static record and the Fit/BalancedAllocation columns
//                      (every load of a node issued before any use, no
//                      data-dependent branches), keeps the packed result of
//                      each of its KN nodes in registers, reduces (DPP + LDS),
//                      normalises from the registers, takes the argmax and the
//                      lane that owns the selected node assumes the pod.
//
// Node n of a replica is owned by workgroup (n / BLOCK) mod S of the replica's
// group and lane n mod BLOCK for every pod, so a node's mutable columns are
// only ever read and written by one lane: an assume needs no barrier.  With
// many replicas S = 1 (config 4: 1,024 replicas fill the chip); with few
// replicas of a large cluster (config 5: 64 replicas x 100,000 nodes, or 8 per
// GPU of an 8-GPU sweep) the S workgroups of a replica exchange their partial
// reductions through per-workgroup slots and a group barrier, two per pod.
// Results equal ksg_queue_kernel's bit for bit (same plugin arithmetic, same
// reductions), which the GPU tests check against the oracle.

// static record layout: kSr* in ksched_kernels.h

struct SweepSlot {          // one workgroup's partials of the current pod (S > 1)
  uint32_t nfeas;
  int32_t minidx, mt, ma;
  uint64_t best;
  uint32_t err;
  int32_t pad;
};

struct SweepArgs {
  int32_t coop;                 // host: launch cooperatively (MULTI instances)
  DevCluster c;
  DevState st;                  // replica r's arrays at base + r * stride
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* profiles;  // [R]
  int32_t b0, nb;               // batch = pods [b0, b0 + nb)
  int32_t out0, count;          // placements[r * count + out0 + j]
  uint64_t* srec;               // [nb][N] static records
  uint64_t* scratch;            // KN == 0 only: [R][N] packed per-node results
  int32_t* placements;
  int32_t S;                    // workgroups per replica (>= 1)
  SweepSlot* slots;             // S > 1: [2][R * S] partials by pod parity
  unsigned* gbar;               // S > 1: [R][16] arrival counters (one 64-B line each), zeroed before the launch
  unsigned* timeout;            // S > 1: set when a group barrier poll gave up
  // narrow state (NARROW instances; ranges checked by the host and by
  // ksg_narrow_init): per node one 16-byte static record {alloc cpu milli,
  // alloc memory MiB, allowed pods, alloc of column nx} and per (replica, node)
  // one 16-byte mutable record {requested cpu milli (EX: 24 bits | requested
  // nx << 24), non-zero cpu milli, requested memory MiB, non-zero memory MiB
  // (24 bits) | pod count << 24}
  const int4* nstat;            // [N]
  const double2* nrcp;          // [N] ddiv_rcp of the cpu / memory MiB allocatable (DevCluster::rcp64)
  int4* nmut;                   // [R][N]
  int32_t nx;                   // EX: the one scalar column any pod of the run requests
};

// Memory in MiB: exact for the Fit and BalancedAllocation arithmetic when every
// memory quantity is a multiple of 2^20 (quotients of equally scaled integers
// are unchanged; float64 quotients of values scaled by a power of two are
// bit-identical), which the host checks.
constexpr int kNarrowMemShift = 20;

// Hand-offs between co-resident workgroups of one launch without cache
// maintenance (MI355X guide, Guideline 16, "Valid forms" row 1): every byte
// another workgroup reads is written with an agent-scope (sc1,
// write-through) store or an agent-scope atomic and read with an agent-scope
// global (sc1) load; every storing wave drains before the workgroup barrier in
// front of the one-lane arrival; the poll is an sc1 load; the other waves
// load after the workgroup barrier the polling lane joins.  No release
// (buffer_wbl2) and no acquire (buffer_inv).  Used by the multi-workgroup
// replica sweep and the chip-wide topology path.
template <class T>
__device__ __forceinline__ T gld(const T* p) {   // agent-scope (sc1) global load
  return __hip_atomic_load((__attribute__((address_space(1))) T*)(const_cast<T*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
template <class T, class V>
__device__ __forceinline__ void gst(T* p, V v) {   // agent-scope (sc1, write-through) global store
  __hip_atomic_store((__attribute__((address_space(1))) T*)p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void gadd(int32_t* p, int32_t v) {   // agent-scope global atomic add
  __hip_atomic_fetch_add((__attribute__((address_space(1))) int32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gor(int32_t* p, int32_t v) {    // agent-scope global atomic or
  __hip_atomic_fetch_or((__attribute__((address_space(1))) int32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival counter shared by G workgroups (monotonic: the k-th barrier
// completes at k * G); the poll is bounded and a timeout is reported.
__device__ __forceinline__ bool arrive_and_wait_sc1(unsigned* bar, unsigned* timeout, int G, unsigned& target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 stores and atomics are done
  __syncthreads();
  target += (unsigned)G;
  __shared__ int s_timeout;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)bar, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int to = 0;
    while (gld(bar) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 26) || gld(timeout)) {
        gst(timeout, 1u);
        to = 1;
        break;
      }
    }
    s_timeout = to;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler ordering only: loads stay below the poll
  __syncthreads();
  return s_timeout == 0;
}

// 1-D grid of static_blocks(N, nb) workgroups.  XCD-aware order (MI355X guide
// T1, speed only): workgroups b and b + 8 share an XCD, so every pod of one
// node tile lands in the same group of 8 and the tile's static columns are
// read from HBM once per launch and from that XCD's L2 for the other pods
// (config 5: 64 taints + 50 images per node, ~0.5 KB, re-read by 64 pods).
__host__ __device__ inline int static_tiles8(int N) { return ((N + 255) / 256 + 7) / 8 * 8; }
__host__ __device__ inline int static_blocks(int N, int nb) { return static_tiles8(N) * nb; }

// The node's taint slots in chunks of kStaticChunk independent loads (the
// slot loops of untolerated_slot / taint_score end at the first empty slot and
// chain every load behind the previous compare): TaintToleration's Filter
// verdict (an untolerated NoSchedule / NoExecute taint) and its Score count
// (untolerated PreferNoSchedule taints) in one pass; effects from LDS.
constexpr int kStaticChunk = 8;
constexpr int kStaticEff = 4096;   // taint vocabulary staged in LDS up to this size

__device__ __forceinline__ void static_taints(const DevCluster& c, int n, const int32_t* tolf, const int32_t* tolp,
                                              const uint8_t* eff, bool& reject, int64_t& score, int* slot = nullptr) {
  reject = false;
  score = 0;
  int first = -1;   // untolerated_slot: the first rejecting slot
  for (int s0 = 0; s0 < c.T; s0 += kStaticChunk) {
    uint32_t id[kStaticChunk];
#pragma unroll
    for (int k = 0; k < kStaticChunk; k++) id[k] = s0 + k < c.T ? c.taints[(size_t)(s0 + k) * c.N + n] : 0u;
    bool end = false;
#pragma unroll
    for (int k = 0; k < kStaticChunk; k++) {
      end |= id[k] == 0;
      if (end) continue;
      const uint32_t vid = id[k] - 1;
      const uint8_t e = eff[vid];
      if (e == KSG_EFFECT_NO_SCHEDULE || e == KSG_EFFECT_NO_EXECUTE) {
        const bool r = !tol_bit(tolf, vid);
        if (r && first < 0) first = s0 + k;
        reject |= r;
      } else if (e == KSG_EFFECT_PREFER_NO_SCHEDULE) {
        score += !tol_bit(tolp, vid);
      }
    }
    if (end) break;
  }
  if (slot) *slot = first;
}

// ImageLocality's sum over the pod's image entries, the node's sorted image
// ids read in chunks of independent loads (image_score's arithmetic after it).
__device__ __forceinline__ int64_t static_images(const DevCluster& c, int n, const int32_t* P, int img,
                                                 int n_containers) {
  int64_t sum = 0;
  if (img >= 0) {
    const int32_t* w0 = P + img;
    const int cnt = *w0++;
    uint32_t top = 0;   // largest image id the pod asks for
    for (int i = 0; i < cnt; i++) top = max(top, (uint32_t)w0[3 * i]);
    for (int s0 = 0; cnt > 0 && s0 < c.I; s0 += kStaticChunk) {
      uint32_t x[kStaticChunk];
#pragma unroll
      for (int k = 0; k < kStaticChunk; k++) x[k] = s0 + k < c.I ? c.images[(size_t)(s0 + k) * c.N + n] : 0u;
      bool end = false;
#pragma unroll
      for (int k = 0; k < kStaticChunk; k++) {
        end |= x[k] == 0 || x[k] > top;
        if (end) continue;
        for (int i = 0; i < cnt; i++)
          if ((uint32_t)w0[3 * i] == x[k]) sum += ld64(w0 + 3 * i + 1);
      }
      if (end) break;
    }
  }
  const int64_t mb = 1024 * 1024, minT = 23 * mb;
  const int64_t mx = 1000 * mb * (int64_t)n_containers;
  if (sum < minT) sum = minT;
  else if (sum > mx) sum = mx;
  return div_small(100 * (sum - minT), mx - minT);
}

// The static record of (pod, node n): the replica-independent verdicts and raw
// scores (also computed in place by ksg_topo_coop's one-pod evaluation).
__device__ __forceinline__ uint64_t static_record(const DevCluster& c, const ksg_pod& p, const PodView& v, int n,
                                                  const uint8_t* eff) {
  const GNode nd{&c, n};
  uint32_t bits = 0;
  if (v.reject || (v.node_set && !((((uint32_t)v.node_set[n >> 5]) >> (n & 31)) & 1u))) bits |= kSrNotEval;
  if (nd.unsched() && !(p.flags & KSG_POD_TOL_UNSCHED)) bits |= kSrUnsched;
  if (p.node_name != -1 && p.node_name != n) bits |= kSrNodeName;
  bool treject;
  int64_t tscore;
  int tslot = -1;
  static_taints(c, n, v.tolf, v.tolp, eff, treject, tscore, &tslot);
  if (treject) bits |= kSrTaint;
  if (!na_required_match(nd, v.P, v.na_req)) bits |= kSrNodeAff;
  const uint64_t rt = (uint64_t)tscore;
  const uint64_t ra = v.na_pref >= 0 ? (uint64_t)na_pref_score(nd, v.P, v.na_pref) : 0;
  const uint64_t im = (uint64_t)static_images(c, n, v.P, v.img, p.n_containers);
  return bits | ((rt & 0xff) << 8) | ((ra & 0xffff) << 16) | ((im & 0xff) << 32) |
         ((uint64_t)(tslot < 0 ? 0 : tslot & 0xffff) << kSrTaintSlotShift);
}

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_sweep_static(SweepArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ uint8_t s_eff[kStaticEff];
  const int tid = threadIdx.x;
  const DevCluster& c = a.c;
  const int N = c.N;
  const int b = blockIdx.x, w = b >> 3;
  const int j = w % a.nb;                       // pod of the batch
  const int tile = (w / a.nb) * 8 + (b & 7);    // node tile: same b % 8 for all its pods
  if (tile * 256 >= N) return;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.profiles)[i_];
  const bool eff_lds = c.V <= kStaticEff;
  if (eff_lds)
    for (int i = tid; i < c.V; i += 256) s_eff[i] = c.taint_effect[i];
  stage_pod<256>(a.pods, a.prog, a.b0 + j, &s_pod, s_blob);
  __syncthreads();
  const ksg_pod& p = s_pod;
  const PodView v = make_view(c, s_prof, p, s_blob, a.prog);
  const int n = tile * 256 + tid;
  if (n >= N) return;
  a.srec[(size_t)j * N + n] = static_record(c, p, v, n, eff_lds ? s_eff : c.taint_effect);
}
#endif  // KSG_PART

// Replica-uniform facts of a profile for the sweep.
struct SweepProf {
  bool f_unsched, f_nodename, f_taint, f_na, f_fit;   // filter enabled
  CmProf cm;     // Fit over {cpu, memory} (+ ex), BalancedAllocation over {cpu, memory}
  int ex;        // a third, scalar Fit column (config 5: amd.com/gpu), -1 if none
  int64_t w_ex;
};

// The "fast" sweep arithmetic covers Fit over exactly {cpu, memory} or
// {cpu, memory, one scalar column} with positive weights, and
// BalancedAllocation over exactly {cpu, memory}; sweep_fast_profile() is the
// host mirror.
__device__ __forceinline__ SweepProf sweep_prof(const ksg_profile& prof) {
  SweepProf s{};
  for (int k = 0; k < prof.n_filter; k++) {
    const int pl = prof.filter_order[k];
    s.f_unsched |= pl == KSG_PL_NODE_UNSCHEDULABLE;
    s.f_nodename |= pl == KSG_PL_NODE_NAME;
    s.f_taint |= pl == KSG_PL_TAINT_TOLERATION;
    s.f_na |= pl == KSG_PL_NODE_AFFINITY;
    s.f_fit |= pl == KSG_PL_NODE_RESOURCES_FIT;
  }
  s.cm = cm_prof(prof);
  s.ex = -1;
  s.w_ex = 0;
  if (!s.cm.fast && prof.fit_n == 3 && prof.fit_strategy != KSG_REQUESTED_TO_CAPACITY_RATIO) {
    for (int i = 0; i < 3; i++) {
      const int r = prof.fit_res[i];
      if (r == KSG_RES_CPU) s.cm.wc = prof.fit_w[i];
      else if (r == KSG_RES_MEM) s.cm.wm = prof.fit_w[i];
      else { s.ex = r; s.w_ex = prof.fit_w[i]; }
    }
  }
  return s;
}

// Pod-uniform values of one replica's evaluation of pod p.
struct SweepPod {
  uint32_t fmask;      // static-record bits that reject
  bool fit_on;
  bool ex_on;          // Fit scores the scalar column sp.ex (the pod requests it)
  uint32_t req_mask;   // resource columns the Fit filter checks
  int64_t w_fit, w_ba, w_img, w_t, w_a;
  uint32_t smask;
};

__device__ __forceinline__ SweepPod sweep_pod(const SweepProf& sp, const ksg_profile& prof, const ksg_pod& p, int R) {
  SweepPod q;
  const uint32_t fs = p.filter_skip;
  auto on = [&](bool en, int pl) { return en && !((fs >> pl) & 1u); };
  q.fmask = kSrNotEval | (on(sp.f_unsched, KSG_PL_NODE_UNSCHEDULABLE) ? kSrUnsched : 0u) |
            (on(sp.f_nodename, KSG_PL_NODE_NAME) ? kSrNodeName : 0u) |
            (on(sp.f_taint, KSG_PL_TAINT_TOLERATION) ? kSrTaint : 0u) |
            (on(sp.f_na, KSG_PL_NODE_AFFINITY) ? kSrNodeAff : 0u);
  q.fit_on = on(sp.f_fit, KSG_PL_NODE_RESOURCES_FIT);
  q.ex_on = sp.ex >= 0 && p.req[sp.ex] > 0;   // alloc_req: a scalar the pod does not request is skipped
  uint32_t m = 0;
  for (int r = 0; r < R && r < KSG_MAX_RES; r++)
    if (p.req[r] > 0 && !(r >= 3 && ((prof.fit_ignored_res >> r) & 1u))) m |= 1u << r;
  q.req_mask = m;
  q.smask = prof.score_mask & ~p.score_skip & ~(bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD));
  auto w = [&](int pl) { return (q.smask & bit(pl)) ? (int64_t)prof.weight[pl] : (int64_t)0; };
  q.w_fit = w(KSG_PL_NODE_RESOURCES_FIT);
  q.w_ba = w(KSG_PL_BALANCED_ALLOCATION);
  q.w_img = w(KSG_PL_IMAGE_LOCALITY);
  q.w_t = w(KSG_PL_TAINT_TOLERATION);
  q.w_a = w(KSG_PL_NODE_AFFINITY);
  return q;
}

// The pod's cpu / memory requests in the units of the columns (memory in MiB
// on the narrow instances).
struct PodCM {
  int64_t req_c, req_m, nz_c, nz_m;
};

template <bool NARROW>
__device__ __forceinline__ PodCM pod_cm(const ksg_pod& p) {
  if constexpr (NARROW)
    return PodCM{p.req[KSG_RES_CPU], p.req[KSG_RES_MEM] >> kNarrowMemShift, p.nz_cpu, p.nz_mem >> kNarrowMemShift};
  else
    return PodCM{p.req[KSG_RES_CPU], p.req[KSG_RES_MEM], p.nz_cpu, p.nz_mem};
}

// Fit (cpu + memory [+ ex]) and BalancedAllocation (cpu + memory) scores from
// loaded values: fit_score / ba_score restated without branches (cm_scores'
// arithmetic).  ex_on: Fit also scores the scalar column with allocatable ae,
// requested re, pod request qx and weight w_ex.
__device__ __forceinline__ void sweep_cm_scores(const CmProf& m, const PodCM& p, int64_t ac, int64_t am, int64_t rc,
                                                int64_t rm, int64_t zc, int64_t zm, bool ex_on, int64_t ae,
                                                int64_t re, int64_t qx, int64_t w_ex, int64_t& fit, int64_t& ba) {
  const bool hc = ac > 0, hm = am > 0;
  const int64_t sac = hc ? ac : 1, sam = hm ? am : 1;
  const float ic = __builtin_amdgcn_rcpf((float)sac), im = __builtin_amdgcn_rcpf((float)sam);
  const int64_t qc = zc + p.nz_c, qm = zm + p.nz_m;
  int64_t xc, xm;
  if (m.least) {
    xc = qc > ac ? 0 : (ac - qc) * 100;
    xm = qm > am ? 0 : (am - qm) * 100;
  } else {
    xc = (qc > ac ? ac : qc) * 100;
    xm = (qm > am ? am : qm) * 100;
  }
  const int64_t sc = qdiv(xc, sac, ic), sm = qdiv(xm, sam, im);
  int64_t num = (hc ? sc * m.wc : 0) + (hm ? sm * m.wm : 0);
  int64_t ws = (hc ? m.wc : 0) + (hm ? m.wm : 0);
  if (ex_on) {
    const bool he = ae > 0;
    const int64_t sae = he ? ae : 1, qe = re + qx;
    const int64_t xe = m.least ? (qe > ae ? 0 : (ae - qe) * 100) : (qe > ae ? ae : qe) * 100;
    const int64_t se = qdiv(xe, sae, __builtin_amdgcn_rcpf((float)sae));
    num += he ? se * w_ex : 0;
    ws += he ? w_ex : 0;
  }
  fit = ws == 0 ? 0 : qdiv(num, ws, __builtin_amdgcn_rcpf((float)ws));
  const double dac = (double)sac, dam = (double)sam;
  double fc = ddiv((double)(rc + p.req_c), dac);
  double fm = ddiv((double)(rm + p.req_m), dam);
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = hc && hm ? fabs((fc - fm) / 2) : 0.0;
  ba = (int32_t)((1 - sd) * (double)100);
}

// sweep_cm_scores on the narrow records, in 32-bit integers: the range checks
// (narrow_candidate, ksg_narrow_init) bound every product below 2^30, so the
// quotients equal the int64 ones; BalancedAllocation's float64 quotients use
// the per-node reciprocals (ddiv_r: the same bits as ddiv).
__device__ __forceinline__ void sweep_cm_scores32(const CmProf& m, const PodCM& p, int32_t ac, int32_t am,
                                                  int32_t rc, int32_t rm, int32_t zc, int32_t zm, double2 rcp,
                                                  bool ex_on, int32_t ae, int32_t re, int32_t qx, int32_t w_ex,
                                                  int64_t& fit, int64_t& ba) {
  const bool hc = ac > 0, hm = am > 0;
  const int32_t sac = hc ? ac : 1, sam = hm ? am : 1;
  const float ic = __builtin_amdgcn_rcpf((float)sac), im = __builtin_amdgcn_rcpf((float)sam);
  const int32_t qc = zc + (int32_t)p.nz_c, qm = zm + (int32_t)p.nz_m;
  int32_t xc, xm;
  if (m.least) {
    xc = qc > ac ? 0 : (ac - qc) * 100;
    xm = qm > am ? 0 : (am - qm) * 100;
  } else {
    xc = (qc > ac ? ac : qc) * 100;
    xm = (qm > am ? am : qm) * 100;
  }
  const int32_t sc = qdiv32(xc, sac, ic), sm = qdiv32(xm, sam, im);
  const int32_t wc = (int32_t)m.wc, wm = (int32_t)m.wm;
  int32_t num = (hc ? sc * wc : 0) + (hm ? sm * wm : 0);
  int32_t ws = (hc ? wc : 0) + (hm ? wm : 0);
  if (ex_on) {
    const bool he = ae > 0;
    const int32_t sae = he ? ae : 1, qe = re + qx;
    const int32_t xe = m.least ? (qe > ae ? 0 : (ae - qe) * 100) : (qe > ae ? ae : qe) * 100;
    const int32_t se = qdiv32(xe, sae, __builtin_amdgcn_rcpf((float)sae));
    num += he ? se * w_ex : 0;
    ws += he ? w_ex : 0;
  }
  fit = ws == 0 ? 0 : qdiv32(num, ws, __builtin_amdgcn_rcpf((float)ws));
  double fc = ddiv_r((double)(rc + (int32_t)p.req_c), (double)sac, rcp.x);
  double fm = ddiv_r((double)(rm + (int32_t)p.req_m), (double)sam, rcp.y);
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = hc && hm ? fabs((fc - fm) / 2) : 0.0;
  ba = (int32_t)((1 - sd) * (double)100);
}

struct OpMaxI32 { __device__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; } };

struct SweepPart {
  uint32_t nfeas;
  int32_t minidx, mt, ma;
};

// KN > 0: the lane's nodes are base + k * S * BLOCK, k < KN (base = sub * BLOCK +
// tid), results kept in registers.  KN == 0: the same nodes for k while < N,
// results in the replica's scratch row.
// FAST: every replica's Fit and BalancedAllocation score exactly {cpu, memory}
// with positive weights (CmProf::fast; the host checks it for all replicas);
// otherwise the generic plugin arithmetic on the loaded columns.
// MULTI: S > 1 workgroups per replica (runtime stride S * BLOCK between a
// lane's nodes); without it S == 1 and the stride is the constant BLOCK, which
// keeps the node offsets in the load instructions' immediates.
// EX (with FAST): some replica's Fit also scores one scalar column (SweepProf::ex).
// NARROW (with FAST): the 16-byte static and mutable records above instead of
// the int64 columns (16 instead of 36 bytes of per-replica state per (replica,
// pod, node)); the pods of the run request nothing beyond cpu, memory and
// (EX) column a.nx.
template <int BLOCK, int KN, bool FAST, bool MULTI, bool EX = false, bool NARROW = false>
__global__ __launch_bounds__(BLOCK, 1024 / BLOCK) void ksg_sweep(SweepArgs a) {   // 16 waves per CU
  static_assert(!NARROW || FAST, "narrow state: the fast cpu/memory arithmetic");
  constexpr int NW = BLOCK / 64;
  // nodes whose loads are in flight together (narrow: 40 B per node, room for 4)
  constexpr int U = !FAST ? (KN == 0 ? 2 : 1) : (NARROW && KN == 0 ? 4 : (KN >= 20 || EX ? 2 : 4));
  __shared__ ksg_profile s_prof;
  __shared__ SweepPart s_part[2][NW];
  __shared__ uint64_t s_best[2][NW];
  __shared__ uint32_t s_err[2][NW];
  __shared__ SweepPart s_grp[2];        // S > 1: the replica's totals
  __shared__ uint64_t s_gbest[2];
  __shared__ uint32_t s_gerr[2];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int S = MULTI ? a.S : 1;
  const int rep = MULTI ? blockIdx.x / S : blockIdx.x, sub = MULTI ? blockIdx.x - rep * S : 0;
  const int stride = MULTI ? S * BLOCK : BLOCK;   // between a lane's nodes
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  const size_t NN = (size_t)N;
  int64_t* requested = a.st.requested + rep * a.st.stride_req;
  int64_t* nonzero = a.st.nonzero + rep * a.st.stride_nz;
  int32_t* pod_count = a.st.pod_count + rep * a.st.stride_pc;
  int4* nmut = NARROW ? a.nmut + (size_t)rep * N : nullptr;
  uint64_t* scratch = KN == 0 ? a.scratch + (size_t)rep * N : nullptr;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.profiles + rep)[i_];
  __syncthreads();
  const ksg_profile& prof = s_prof;
  const SweepProf sp = sweep_prof(prof);
  constexpr int KR = KN > 0 ? KN : 1;
  uint64_t recs[KR];
  unsigned target = 0;
  const size_t slot_base = (size_t)rep * S;   // this replica's slots within a parity set

  for (int j = 0; j < a.nb; j++) {
    const ksg_pod& p = a.pods[a.b0 + j];
    const SweepPod q = sweep_pod(sp, prof, p, R);
    const PodCM pc4 = pod_cm<NARROW>(p);
    const int32_t qx32 = EX && NARROW ? (int32_t)p.req[a.nx] : 0;
    const uint64_t* srec = a.srec + (size_t)j * N;
    const int par = j & 1;
    SweepSlot* slots = a.slots + (size_t)par * gridDim.x;

    // ---- sweep A: filters + raw scores of this lane's nodes ------------------
    uint32_t nfeas = 0;
    int32_t minidx = 0x7fffffff, mt = 0, ma = 0;
    auto feasible = [&](int n, uint64_t sr, const NodeCols& L) {
      bool ok = (sr & q.fmask) == 0;
      if (q.fit_on) ok = ok && fit_filter(c, p, L, prof.fit_ignored_res) == 0;
      return ok;
    };
    auto eval_fast = [&](int n, uint64_t sr, int64_t ac, int64_t am, int64_t rc, int64_t rm, int64_t zc, int64_t zm,
                         int32_t pc, int32_t al, int64_t ae, int64_t re, double2 rcp) -> uint64_t {
      bool ok = (sr & q.fmask) == 0;
      if (q.fit_on) {
        ok = ok && pc + 1 <= al;
        ok = ok && (!(q.req_mask & 1u) || pc4.req_c <= ac - rc);
        ok = ok && (!(q.req_mask & 2u) || pc4.req_m <= am - rm);
        if constexpr (NARROW) {
          if (EX && ((q.req_mask >> a.nx) & 1u)) ok = ok && p.req[a.nx] <= ae - re;
        } else {
          for (int r = 2; r < R && r < KSG_MAX_RES; r++)   // pod-uniform: loads only for requested columns
            if ((q.req_mask >> r) & 1u) ok = ok && p.req[r] <= c.alloc[r * NN + n] - requested[r * NN + n];
        }
      }
      if (!ok) return 0;
      int64_t fs = 0, bs = 0;
      if constexpr (NARROW)
        sweep_cm_scores32(sp.cm, pc4, (int32_t)ac, (int32_t)am, (int32_t)rc, (int32_t)rm, (int32_t)zc, (int32_t)zm,
                          rcp, EX && q.ex_on, (int32_t)ae, (int32_t)re, qx32, (int32_t)sp.w_ex, fs, bs);
      else
        sweep_cm_scores(sp.cm, pc4, ac, am, rc, rm, zc, zm, EX && q.ex_on, ae, re, EX ? p.req[EX ? sp.ex : 0] : 0,
                        sp.w_ex, fs, bs);
      const int64_t rt = (sr >> 8) & 0xff, ra = (sr >> 16) & 0xffff, im = (sr >> 32) & 0xff;
      const int64_t part = im * q.w_img + ((q.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) ? fs * q.w_fit : 0) +
                           ((q.smask & bit(KSG_PL_BALANCED_ALLOCATION)) ? bs * q.w_ba : 0);
      return pack_rec(part, rt, ra);
    };
    auto eval_generic = [&](int n, uint64_t sr, const NodeCols& L) -> uint64_t {
      if (!feasible(n, sr, L)) return 0;
      const int64_t fs = fit_score(prof, p, L), bs = ba_score(prof, p, L);
      const int64_t rt = (sr >> 8) & 0xff, ra = (sr >> 16) & 0xffff, im = (sr >> 32) & 0xff;
      const int64_t part = im * q.w_img + ((q.smask & bit(KSG_PL_NODE_RESOURCES_FIT)) ? fs * q.w_fit : 0) +
                           ((q.smask & bit(KSG_PL_BALANCED_ALLOCATION)) ? bs * q.w_ba : 0);
      return pack_rec(part, rt, ra);
    };
    auto account = [&](int n, uint64_t x) {
      if (x >> 63) {
        nfeas += 1;
        minidx = min(minidx, n);
        mt = max(mt, (int32_t)((x >> 48) & 0xff));
        ma = max(ma, (int32_t)((x >> 32) & 0xffff));
      }
    };
    const int iters = KN > 0 ? KN : (N + stride - 1) / stride;
    // opaque per pod: keeps the per-node addresses from being hoisted out of
    // the pod loop (KN x 9 live 64-bit pointers would not fit the VGPR budget)
    int tb = sub * BLOCK + tid;
    asm volatile("" : "+v"(tb));
    auto group = [&](const int k0) {
      if constexpr (FAST) {
        uint64_t sr[U];
        int64_t ac[U], am[U], rc[U], rm[U], zc[U], zm[U], ae[U], re[U];
        int32_t pc[U], al[U];
        double2 rcp[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int n = tb + (k0 + u) * stride;
          const int nl = n < N ? n : 0;   // clamped: every lane loads from a valid address
          sr[u] = srec[nl];
          if constexpr (NARROW) {
            const int4 st4 = a.nstat[nl], mu = nmut[nl];
            rcp[u] = a.nrcp[nl];
            ac[u] = st4.x;
            am[u] = st4.y;
            al[u] = st4.z;
            rc[u] = EX ? (int64_t)((uint32_t)mu.x & 0xffffffu) : (int64_t)mu.x;
            zc[u] = mu.y;
            rm[u] = mu.z;
            zm[u] = (int64_t)((uint32_t)mu.w & 0xffffffu);
            pc[u] = (int32_t)((uint32_t)mu.w >> 24);
            ae[u] = EX ? st4.w : 0;
            re[u] = EX ? (int64_t)((uint32_t)mu.x >> 24) : 0;
          } else {
            ac[u] = c.alloc[KSG_RES_CPU * NN + nl];
            am[u] = c.alloc[KSG_RES_MEM * NN + nl];
            rc[u] = requested[KSG_RES_CPU * NN + nl];
            rm[u] = requested[KSG_RES_MEM * NN + nl];
            zc[u] = nonzero[nl];
            zm[u] = nonzero[NN + nl];
            pc[u] = pod_count[nl];
            al[u] = c.allowed[nl];
            rcp[u] = double2{0.0, 0.0};
          }
          if constexpr (!NARROW) {
            ae[u] = 0;
            re[u] = 0;
          }
          if constexpr (EX && !NARROW) {
            if (q.ex_on) {
              ae[u] = c.alloc[(size_t)sp.ex * NN + nl];
              re[u] = requested[(size_t)sp.ex * NN + nl];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int n = tb + (k0 + u) * stride;
          uint64_t x = 0;
          if (k0 + u < iters && n < N)
            x = eval_fast(n, sr[u], ac[u], am[u], rc[u], rm[u], zc[u], zm[u], pc[u], al[u], ae[u], re[u], rcp[u]);
          account(n, x);
          if constexpr (KN > 0) {
            if (k0 + u < KN) recs[k0 + u < KR ? k0 + u : 0] = x;
          } else {
            if (n < N) scratch[n] = x;
          }
        }
      } else {   // U nodes' records and every resource column in flight
        uint64_t sr[U];
        NodeCols L[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int n = tb + (k0 + u) * stride;
          const int nl = n < N ? n : 0;
          sr[u] = srec[nl];
          load_cols(c, requested, nonzero, pod_count, nl, L[u]);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int n = tb + (k0 + u) * stride;
          uint64_t x = 0;
          if (k0 + u < iters && n < N) x = eval_generic(n, sr[u], L[u]);
          account(n, x);
          if constexpr (KN > 0) {
            if (k0 + u < KN) recs[k0 + u < KR ? k0 + u : 0] = x;
          } else {
            if (n < N) scratch[n] = x;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // one group's loads in flight at a time (register budget)
    };
    if constexpr (KN > 0) {
#pragma unroll
      for (int k0 = 0; k0 < KN; k0 += U) group(k0);
    } else {
      for (int k0 = 0; k0 < iters; k0 += U) group(k0);
    }
    {
      SweepPart w;
      w.nfeas = wreduce(nfeas, OpAdd32{});
      w.minidx = wreduce(minidx, OpMin32{});
      w.mt = wreduce(mt, OpMaxI32{});
      w.ma = wreduce(ma, OpMaxI32{});
      if (lane == 0) s_part[par][wv] = w;
    }
    __syncthreads();
    uint32_t gn = 0;
    int32_t gmin = 0x7fffffff, gmt = 0, gma = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const SweepPart w = s_part[par][i];
      gn += w.nfeas;
      gmin = min(gmin, w.minidx);
      gmt = max(gmt, w.mt);
      gma = max(gma, w.ma);
    }
    if (MULTI) {   // the replica's totals over its S workgroups
      if (tid == 0) {
        SweepSlot& o = slots[slot_base + sub];   // sc1 stores: the fence-free hand-off (arrive_and_wait_sc1)
        gst(&o.nfeas, gn);
        gst(&o.minidx, gmin);
        gst(&o.mt, gmt);
        gst(&o.ma, gma);
      }
      if (!arrive_and_wait_sc1(a.gbar + 16 * rep, a.timeout, S, target)) return;
      if (wv == 0) {
        uint32_t n_ = 0;
        int32_t mi = 0x7fffffff, t_ = 0, a_ = 0;
        for (int qi = lane; qi < S; qi += 64) {
          const SweepSlot* o = slots + slot_base + qi;
          n_ += gld(&o->nfeas);
          mi = min(mi, gld(&o->minidx));
          t_ = max(t_, gld(&o->mt));
          a_ = max(a_, gld(&o->ma));
        }
        n_ = wreduce(n_, OpAdd32{});
        mi = wreduce(mi, OpMin32{});
        t_ = wreduce(t_, OpMaxI32{});
        a_ = wreduce(a_, OpMaxI32{});
        if (lane == 0) s_grp[par] = SweepPart{n_, mi, t_, a_};
      }
      __syncthreads();
      gn = s_grp[par].nfeas;
      gmin = s_grp[par].minidx;
      gmt = s_grp[par].mt;
      gma = s_grp[par].ma;
    }
    int selected = -1;
    if (gn == 1) {
      selected = gmin;
    } else if (gn >= 2) {
      // ---- sweep B: normalise, weight, argmax (registers only) ---------------
      const float inv_t = gmt ? __builtin_amdgcn_rcpf((float)gmt) : 1.0f;
      const float inv_a = gma ? __builtin_amdgcn_rcpf((float)gma) : 1.0f;
      uint64_t best = 0;
      uint32_t err = 0;
      auto score = [&](int n, uint64_t x) {
        if (!(x >> 63)) return;
        const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
        int64_t total = part;
        if (q.smask & bit(KSG_PL_TAINT_TOLERATION)) {   // 100 * rt < 2^15, 100 * ra < 2^23: qdiv32's range
          const int64_t s = gmt != 0 ? 100 - (NARROW ? qdiv32(100 * (int32_t)rt, gmt, inv_t) : qdiv(100 * rt, gmt, inv_t)) : 100;
          err |= (s < 0 || s > 100);
          total += s * q.w_t;
        }
        if (q.smask & bit(KSG_PL_NODE_AFFINITY)) {
          const int64_t s = gma != 0 ? (NARROW ? qdiv32(100 * (int32_t)ra, gma, inv_a) : qdiv(100 * ra, gma, inv_a)) : ra;
          err |= (s < 0 || s > 100);
          total += s * q.w_a;
        }
        const uint64_t key = argmax_key(total, n);
        best = key > best ? key : best;
      };
      if constexpr (KN > 0) {
#pragma unroll
        for (int k = 0; k < KN; k++) {
          score(tb + k * stride, recs[k]);
          if ((k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
      } else {   // four scratch words in flight per step
        int n = sub * BLOCK + tid;
        for (; n + 3 * stride < N; n += 4 * stride) {
          const uint64_t x0 = scratch[n], x1 = scratch[n + stride], x2 = scratch[n + 2 * stride],
                         x3 = scratch[n + 3 * stride];
          score(n, x0);
          score(n + stride, x1);
          score(n + 2 * stride, x2);
          score(n + 3 * stride, x3);
        }
        for (; n < N; n += stride) score(n, scratch[n]);
      }
      best = wreduce(best, OpMaxU64{});
      err = wreduce(err, OpOr32{});
      if (lane == 0) {
        s_best[par][wv] = best;
        s_err[par][wv] = err;
      }
      __syncthreads();
      uint64_t gb = 0;
      bool gerr = false;
#pragma unroll
      for (int i = 0; i < NW; i++) {
        gb = s_best[par][i] > gb ? s_best[par][i] : gb;
        gerr |= s_err[par][i] != 0;
      }
      if (MULTI) {   // the replica's argmax over its S workgroups
        if (tid == 0) {
          SweepSlot& o = slots[slot_base + sub];
          gst(&o.best, gb);
          gst(&o.err, gerr ? 1u : 0u);
        }
        if (!arrive_and_wait_sc1(a.gbar + 16 * rep, a.timeout, S, target)) return;
        if (wv == 0) {
          uint64_t b_ = 0;
          uint32_t e_ = 0;
          for (int qi = lane; qi < S; qi += 64) {
            const SweepSlot* o = slots + slot_base + qi;
            const uint64_t ob = gld(&o->best);
            b_ = ob > b_ ? ob : b_;
            e_ |= gld(&o->err);
          }
          b_ = wreduce(b_, OpMaxU64{});
          e_ = wreduce(e_, OpOr32{});
          if (lane == 0) { s_gbest[par] = b_; s_gerr[par] = e_; }
        }
        __syncthreads();
        gb = s_gbest[par];
        gerr = s_gerr[par] != 0;
      }
      if (!gerr) selected = key_node(gb);
    }
    // ---- assume: the lane that owns the selected node ------------------------
    if (selected >= 0 && (!MULTI || ((selected / BLOCK) % S) == sub) && (selected % BLOCK) == tid) {
      if constexpr (NARROW) {
        // packed fields: the range checks bound every sum below its field
        int4 mu = nmut[selected];
        mu.x = (int32_t)((uint32_t)mu.x + (uint32_t)pc4.req_c + (EX ? (uint32_t)p.req[a.nx] << 24 : 0u));
        mu.y = (int32_t)((uint32_t)mu.y + (uint32_t)pc4.nz_c);
        mu.z = (int32_t)((uint32_t)mu.z + (uint32_t)pc4.req_m);
        mu.w = (int32_t)((uint32_t)mu.w + (uint32_t)pc4.nz_m + (1u << 24));
        nmut[selected] = mu;
      } else {
        for (int r = 0; r < R; r++) requested[(size_t)r * N + selected] += p.req[r];
        nonzero[selected] += p.nz_cpu;
        nonzero[NN + selected] += p.nz_mem;
        pod_count[selected] += 1;
      }
    }
    if (sub == 0 && tid == 0) a.placements[(size_t)rep * a.count + a.out0 + j] = selected;
  }
}

// Narrow bounds the node side must meet (the pod side is checked on the host):
// per placed pod, at most xc / xm (MiB) of non-zero request beyond its request.
struct NarrowBounds {
  int64_t xc, xm;
  int32_t nx;      // EX column, -1 without
  int32_t places;  // pods a node can still take: min(queue length, 255)
};

// Narrow state of every replica from the int64 columns (every replica starts
// from the context's state): one static record per node, the mutable record
// broadcast.  A node outside the ranges sets *bad; the host then runs the
// int64 instances instead (nothing here writes the context's state).
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_narrow_init(DevCluster c, DevState st, int4* nstat, int4* nmut, int R,
                                                       NarrowBounds b, unsigned* bad) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int N = c.N;
  if (n >= N) return;
  const size_t NN = N;
  constexpr int64_t kMiB = (int64_t)1 << kNarrowMemShift, k24 = (int64_t)1 << 24;
  const int64_t ac = c.alloc[KSG_RES_CPU * NN + n], am = c.alloc[KSG_RES_MEM * NN + n];
  const int64_t rc = st.requested[KSG_RES_CPU * NN + n], rm = st.requested[KSG_RES_MEM * NN + n];
  const int64_t zc = st.nonzero[n], zm = st.nonzero[NN + n];
  const int32_t pc = st.pod_count[n], al = c.allowed[n];
  const int64_t ae = b.nx >= 0 ? c.alloc[(size_t)b.nx * NN + n] : 0;
  const int64_t re = b.nx >= 0 ? st.requested[(size_t)b.nx * NN + n] : 0;
  const int64_t cmax = b.nx >= 0 ? k24 - 1 : (int64_t)INT32_MAX;
  bool ok = ac >= 0 && rc >= 0 && am >= 0 && rm >= 0 && zc >= 0 && zm >= 0 && ae >= 0 && re >= 0;
  ok = ok && ((am | rm | zm) & (kMiB - 1)) == 0;
  ok = ok && ac <= cmax && rc <= cmax;                                   // requested cpu <= max(rc, ac)
  ok = ok && zc + ac + b.places * b.xc <= (int64_t)INT32_MAX;            // Σ placed cpu requests <= ac
  ok = ok && (am >> kNarrowMemShift) <= (int64_t)INT32_MAX && (rm >> kNarrowMemShift) <= (int64_t)INT32_MAX;
  ok = ok && (zm >> kNarrowMemShift) + (am >> kNarrowMemShift) + b.places * b.xm < k24;
  ok = ok && pc >= 0 && pc <= 255 && al >= 0 && al <= 255;              // pod count <= max(pc, al)
  ok = ok && ae <= 255 && re <= 255;
  ok = ok && ac * 100 < (1 << 30) && (am >> kNarrowMemShift) * 100 < (1 << 30);   // sweep_cm_scores32's range
  if (!ok) {
    atomicOr(bad, 1u);
    return;
  }
  const int4 mu = make_int4((int32_t)(rc | (re << 24)), (int32_t)zc, (int32_t)(rm >> kNarrowMemShift),
                            (int32_t)((zm >> kNarrowMemShift) | ((int64_t)pc << 24)));
  if (blockIdx.y == 0) nstat[n] = make_int4((int32_t)ac, (int32_t)(am >> kNarrowMemShift), al, (int32_t)ae);
  for (int r = blockIdx.y; r < R; r += gridDim.y) nmut[(size_t)r * N + n] = mu;
}
#endif  // KSG_PART

// Σ requested cpu / memory per replica from the narrow state (the summaries).
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_narrow_sums(const int4* nmut, int N, uint32_t cpu_mask, int64_t* out) {
  __shared__ int64_t s_p[2][4];
  const int4* q = nmut + (size_t)blockIdx.x * N;
  int64_t a = 0, b = 0;
  for (int n = threadIdx.x; n < N; n += 256) {
    const int4 m = q[n];
    a += (uint32_t)m.x & cpu_mask;
    b += (int64_t)m.z << kNarrowMemShift;
  }
  a = wave_sum64(a);
  b = wave_sum64(b);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { s_p[0][wv] = a; s_p[1][wv] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = s_p[0][0] + s_p[0][1] + s_p[0][2] + s_p[0][3];
    out[2 * blockIdx.x + 1] = s_p[1][0] + s_p[1][1] + s_p[1][2] + s_p[1][3];
  }
}
#endif  // KSG_PART
