// Device side of libksched.so: every kernel and the types they share, in
// namespace ksk.  Included by ksched.hip (the host TU, which also compiles
// every kernel not listed in ksched_parts.h) and by ksched_part.hip, compiled
// once per part (-DKSG_PART=k) with only that part's kernel families: the
// heavy template families (ksg_topo_coop, ksg_sweep) build in parallel
// objects.  Non-template kernels are host-TU only (#ifndef KSG_PART).
#pragma once

#include "ksched_kernels.h"

#define KSG_BATCH_MAX 256

namespace ksk {

#include "ksched_hstore.h"

using namespace ksg;

struct Red {
  int64_t max_t;   // TaintToleration raw max over feasible nodes
  int64_t max_a;   // NodeAffinity raw max
  int32_t nfeas;
  int32_t minidx;
};

struct QueueArgs {
  DevCluster c;
  DevState st;
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* profiles;  // [n_replicas]
  int32_t first, count;
  int32_t do_commit;
  int32_t* placements;          // [n_replicas][count]
  ksg_result* results;          // [n_replicas][count] or null
  uint32_t* cap_fstatus;        // [count][N] or null (replica 0 only)
  int64_t* cap_raw;             // [count][NPLUGINS][N]
  int64_t* cap_norm;
  int64_t* cap_total;           // [count][N]
};

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ksg_queue_kernel(QueueArgs a) {
  constexpr int NW = BLOCK / 64;
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ Red s_red[NW];
  __shared__ uint64_t s_best[NW];
  __shared__ uint32_t s_err[NW];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rep = blockIdx.x;
  const DevCluster& c = a.c;
  const int N = c.N;
  int64_t* requested = a.st.requested + rep * a.st.stride_req;
  int64_t* nonzero = a.st.nonzero + rep * a.st.stride_nz;
  int32_t* pod_count = a.st.pod_count + rep * a.st.stride_pc;
  int32_t* cnt = a.st.cnt + rep * a.st.stride_cnt;
  int32_t* tab = a.st.tab + rep * a.st.stride_tab;
  int32_t* tmpl_total = a.st.tmpl_total + rep * a.st.stride_tt;
  int64_t* partial = a.st.partial + rep * a.st.stride_part;
  int64_t* sraw = a.st.sraw + rep * a.st.stride_sraw;
  uint32_t* ports = a.st.ports ? a.st.ports + rep * a.st.stride_ports : nullptr;
  const bool cap = a.cap_fstatus != nullptr && rep == 0;

  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.profiles + rep)[i_];

  for (int k = 0; k < a.count; k++) {
    const int pi = a.first + k;
    __syncthreads();  // previous pod fully consumed; its commit is visible
    stage_pod<BLOCK>(a.pods, a.prog, pi, &s_pod, s_blob);
    __syncthreads();
    const ksg_pod& p = s_pod;
    const ksg_profile& prof = s_prof;
    const PodView v = make_view(c, prof, p, s_blob, a.prog, false, ports);
    uint32_t* cfs = cap ? a.cap_fstatus + (size_t)k * N : nullptr;
    int64_t* craw = cap ? a.cap_raw + (size_t)k * KSG_NPLUGINS * N : nullptr;
    int64_t* cnorm = cap ? a.cap_norm + (size_t)k * KSG_NPLUGINS * N : nullptr;

    // ---- sweep A: filters + raw scores ------------------------------------
    Red r{0, 0, 0, 0x7fffffff};
    for (int n = tid; n < N; n += BLOCK) {
      const NodeEval e = eval_node(c, prof, v, requested, nonzero, pod_count, n, craw, cnorm);
      if (cap) cfs[n] = e.st;
      if (e.st == 0) {
        r.nfeas += 1;
        r.minidx = min(r.minidx, n);
        r.max_t = max(r.max_t, e.rt);
        r.max_a = max(r.max_a, e.ra);
        sraw[n] = e.rt;
        sraw[(size_t)N + n] = e.ra;
        partial[n] = e.part;
      } else {
        partial[n] = -1;
      }
    }
    {
      Red w;
      w.max_t = wave_max64(r.max_t);
      w.max_a = wave_max64(r.max_a);
      w.nfeas = wave_sum32(r.nfeas);
      w.minidx = wave_min32(r.minidx);
      if (lane == 0) s_red[wv] = w;
    }
    __syncthreads();
    Red g{0, 0, 0, 0x7fffffff};
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const Red w = s_red[i];
      g.max_t = max(g.max_t, w.max_t);
      g.max_a = max(g.max_a, w.max_a);
      g.nfeas += w.nfeas;
      g.minidx = min(g.minidx, w.minidx);
    }

    int selected = -1;
    uint32_t status = 0;
    if (cap && g.nfeas == 1 && tid == 0)   // one feasible node: no Score runs, nothing recorded
      for (int q = 0; q < KSG_NPLUGINS; q++) craw[(size_t)q * N + g.minidx] = cnorm[(size_t)q * N + g.minidx] = 0;
    if (g.nfeas == 1) {
      selected = g.minidx;
    } else if (g.nfeas >= 2) {
      status |= KSG_ST_SCORED;
      // ---- sweep B: normalise, weight, argmax ------------------------------
      uint64_t best = 0;
      uint32_t err = 0;
      int64_t* ctot = cap ? a.cap_total + (size_t)k * N : nullptr;
      for (int n = tid; n < N; n += BLOCK) {
        const int64_t part = partial[n];
        if (part < 0) continue;
        int64_t nt = 0, na = 0;
        const int64_t total = total_score(v, part, sraw[n], sraw[(size_t)N + n], g.max_t, g.max_a, err, &nt, &na);
        if (cap) {
          ctot[n] = total;
          if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) cnorm[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = nt;
          if (v.smask & bit(KSG_PL_NODE_AFFINITY)) cnorm[(size_t)KSG_PL_NODE_AFFINITY * N + n] = na;
        }
        const uint64_t key = argmax_key(total, n);
        best = key > best ? key : best;
      }
      best = wave_max_u64(best);
      err = wave_or32(err);
      if (lane == 0) { s_best[wv] = best; s_err[wv] = err; }
      __syncthreads();
      uint64_t gb = 0;
      uint32_t ge = 0;
#pragma unroll
      for (int i = 0; i < NW; i++) {
        gb = s_best[i] > gb ? s_best[i] : gb;
        ge |= s_err[i];
      }
      if (ge) status |= KSG_ST_SCORE_ERROR;
      else selected = key_node(gb);
    }
    uint32_t score_skip;
    ipa_skip_bits(prof, p, status, score_skip);
    if (tid == 0) {
      if (a.do_commit && selected >= 0)
        commit_node(c, requested, nonzero, pod_count, cnt, tab, tmpl_total, p,
                    v.commit >= 0 ? s_blob + v.commit : nullptr, selected, 1, ports,
                    v.ports >= 0 ? s_blob + v.ports : nullptr);
      a.placements[(size_t)rep * a.count + k] = selected;
      if (a.results) {
        ksg_result res;
        res.selected = selected;
        res.n_feasible = g.nfeas;
        res.status = status;
        res.score_skip = score_skip;
        a.results[(size_t)rep * a.count + k] = res;
      }
    }
  }
}

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (int64_t)__shfl_xor(v, o, 64);
  return v;
}

// ---- batched speculate-and-repair --------------------------------------------
// Phase-1 statistics of pod j of a batch (against the batch-start state).
struct P1Stats {
  int32_t nfeas, minidx;   // feasible nodes, lowest feasible index
  int32_t mt, ma;          // max raw TaintToleration / NodeAffinity score over feasible nodes
  int32_t ht, ha;          // feasible nodes holding mt / ma
  int32_t err;             // some normalised score left [0, 100]
  int32_t K;               // |top set| = min(j + 1, nfeas)
  float inv_mt, inv_ma;    // 1 / mt, 1 / ma (qdiv estimates; 1 when the maximum is 0)
  int32_t pad;
};

struct BatchArgs {
  DevCluster c;
  DevState st;              // replica 0
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* prof;
  int32_t b0, nb;           // batch = pods [b0, b0 + nb)
  int32_t out0;             // output index of pod b0
  int32_t prog_lo, prog_len;  // program range covering the batch's blobs
  unsigned long long* stamps;  // diagnostic build only (KSG_STAMPS): per-segment cycle sums
  uint64_t* rec;            // [KSG_BATCH_MAX][N] packed phase-1 records
  int32_t* img;             // [KSG_BATCH_MAX][N] weight x ImageLocality score of feasible nodes
  int32_t* stat;            // [KSG_BATCH_MAX][N] the slot walk's N32 instances: img + the normalised
                            // TaintToleration / NodeAffinity terms under the phase-1 maxima
                            // (written by top-k), or null
  int32_t* pmax;            // [KSG_BATCH_MAX][2] phase-1 maxima (taint, node affinity)
  P1Stats* p1;              // [KSG_BATCH_MAX]
  uint64_t* top;            // [KSG_BATCH_MAX][KSG_BATCH_MAX] top-set argmax keys
  int32_t* placements;
  ksg_result* results;      // or null
  // pipelined phase 2 (run_pipe): the two-batch window
  int32_t k_extra;          // top sets hold min(j + 1 + k_extra, nfeas) keys
  const int32_t* carry;     // nodes the previous batch changed (slot order), or null
  const int32_t* carry_n;   // their count (device), or null
  int32_t* carry_out;       // this batch's changed nodes, for the next batch
  int32_t* carry_out_n;
  // speculate-and-verify walk (ksched_phase2v.h): phase 1 itself writes the
  // node-major copies rect and imgt ([N][64]: the phase-1 records and weight x
  // ImageLocality) from a 1-D XCD-ordered grid (every pod of a node tile on
  // one XCD, so the partial lines of a node's row merge in that XCD's L2)
  uint64_t* rect;
  int32_t* imgt;
  int32_t xcd_grid;
  // the window pipeline's top-k -> walk hand-off without a cross-stream event
  // (run_pipe): the last top-k workgroup of batch b stores tk_seq = b + 1 into
  // *tk_done; the walk of batch b polls it, then acquires.  Null: stream order.
  unsigned* tk_arrive;      // top-k workgroups of this batch that finished (reset by the last)
  unsigned* tk_done;
  unsigned tk_seq;
  unsigned* tk_timeout;     // set when the walk's poll gave up
  unsigned* walk_err;       // the speculate-and-verify walk's broken-invariant code (armed in every mode)
  int32_t inject_walk_err;  // tests only (env KSG_TEST_INJECT_WALK_ERR): the walk's first item reports code 3
  // the spec walk's hand-off without a release fence (MI355X guide, "valid
  // forms"): top-k stores T and P1Stats with sc0 sc1 stores, every storing
  // wave drains vmcnt(0) before the workgroup barrier in front of the one-lane
  // agent add; the walk loads those bytes with sc0 sc1 loads.  (An agent
  // release per workgroup, buffer_wbl2, made top-k 31 instead of 19 us.)
  int32_t tk_sc;
};

// sc0 sc1 (system-scope relaxed) stores / loads of the spec walk's hand-off bytes
// (global address space explicitly: global_store / global_load, never flat_)
template <typename T>
__device__ __forceinline__ void st_sc(T* p, T v) {
  using GT = __attribute__((address_space(1))) T;
  __hip_atomic_store((GT*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_sc(const T* p) {
  using GT = __attribute__((address_space(1))) T;
  return __hip_atomic_load((GT*)const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// record: bit 63 feasible | rt (8 bits) << 48 | ra (16 bits) << 32 | partial (32 bits)
__device__ __forceinline__ uint64_t pack_rec(int64_t part, int64_t rt, int64_t ra) {
  return (1ull << 63) | ((uint64_t)(rt & 0xff) << 48) | ((uint64_t)(ra & 0xffff) << 32) | (uint32_t)part;
}
__device__ __forceinline__ uint64_t pack_rec(const NodeEval& e) {
  return e.st != 0 ? 0 : pack_rec(e.part, e.rt, e.ra);
}

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_batch_phase1(BatchArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ int32_t s_mt[4], s_ma[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N;
  int j = blockIdx.y, tile = blockIdx.x;
  if (a.xcd_grid) {   // block b: XCD b % 8; all nb pods of tile t run on XCD t % 8
    const int b = blockIdx.x, w = b >> 3;
    j = w % a.nb;
    tile = (w / a.nb) * 8 + (b & 7);
    if (tile * 256 >= N) return;
  }
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.prof)[i_];
  stage_pod<256>(a.pods, a.prog, a.b0 + j, &s_pod, s_blob);
  __syncthreads();
  const PodView v = make_view(c, s_prof, s_pod, s_blob, a.prog);
  const int n = tile * 256 + tid;
  int32_t mt = 0, ma = 0;
  if (n < N) {
    const NodeEval e = eval_node(c, s_prof, v, a.st.requested, a.st.nonzero, a.st.pod_count, n, nullptr, nullptr);
    const uint64_t r = pack_rec(e);
    const int32_t im = e.st == 0 ? (int32_t)e.img : 0;
    a.rec[(size_t)j * N + n] = r;
    a.img[(size_t)j * N + n] = im;
    if (a.imgt) {
      a.rect[(size_t)n * 64 + j] = r;
      a.imgt[(size_t)n * 64 + j] = im;
    }
    if (e.st == 0) { mt = (int32_t)e.rt; ma = (int32_t)e.ra; }
  }
  mt = (int32_t)wave_max64(mt);
  ma = (int32_t)wave_max64(ma);
  if (lane == 0) { s_mt[wv] = mt; s_ma[wv] = ma; }
  __syncthreads();
  if (tid == 0) {
    int32_t bt = 0, ba = 0;
    for (int i = 0; i < 4; i++) { bt = max(bt, s_mt[i]); ba = max(ba, s_ma[i]); }
    if (bt) atomicMax(&a.pmax[2 * j], bt);
    if (ba) atomicMax(&a.pmax[2 * j + 1], ba);
  }
}
#endif  // KSG_PART

// Diagnostic build (-DKSG_STAMPS): lane 0 of wave 0 sums s_memtime deltas per
// segment of the phase-2 loop.  Never compiled into the measured library.
#ifdef KSG_STAMPS
#define KSG_STAMP(seg)                                                   \
  do {                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                   \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();          \
    if (tid == 0) { st_acc[seg] += _t - st_last; st_last = _t; }         \
    __builtin_amdgcn_sched_barrier(0);                                   \
  } while (0)
#else
#define KSG_STAMP(seg) do {} while (0)
#endif

// Phase 1b, one workgroup per pod j: the statistics phase 2 needs to update
// pod j's result incrementally, and the top set T_j = the min(j + 1, nfeas)
// best nodes by (total, lowest index) under the phase-1 maxima.  At most j
// nodes change before pod j, so T_j always contains the best unchanged node.
// The K-th largest key is found by a binary search over a dense key
// ((total - tmin) * N + N - 1 - n), one block count per step.

template <int BLOCK>
__device__ __forceinline__ void batch_topk_body(const BatchArgs& a) {
  constexpr int NW = BLOCK / 64;
  constexpr int kTopQ = 8192 / BLOCK;   // totals held in registers per lane (N <= 8192)
  constexpr long long BIG = 0x7fffffffffffffffll;
  __shared__ ksg_profile s_prof;
  __shared__ long long s_r[NW][4];
  __shared__ int32_t s_i[NW][6];
  __shared__ int32_t s_pos;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = blockIdx.x;
  const DevCluster& c = a.c;
  const int N = c.N;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.prof)[i_];
  if (tid == 0) s_pos = 0;
  __syncthreads();
  const ksg_pod& p = a.pods[a.b0 + j];
  const PodView v = make_view(c, s_prof, p, nullptr, a.prog);
  const int64_t mt = a.pmax[2 * j], ma = a.pmax[2 * j + 1];
  const uint64_t* rec = a.rec + (size_t)j * N;

  int32_t nfeas = 0, minidx = 0x7fffffff, ht = 0, ha = 0;
  uint32_t err = 0;
  int64_t tmin = BIG, tmax = -BIG;
  auto total_of = [&](uint64_t x, uint32_t& e) -> int64_t {
    const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
    return total_score(v, part, rt, ra, mt, ma, e, nullptr, nullptr);
  };
  int64_t tot[kTopQ];
  // the slot walk's N32 instances add Fit + BalancedAllocation to this (the
  // record's partial minus img is exactly those two weighted scores)
  int32_t* stat = a.stat ? a.stat + (size_t)j * N : nullptr;
  const int32_t* img = a.img + (size_t)j * N;
#pragma unroll
  for (int q = 0; q < kTopQ; q++) {
    const int n = tid + q * BLOCK;
    tot[q] = BIG;   // BIG = infeasible
    if (n >= N) continue;
    const uint64_t x = rec[n];
    if (!(x >> 63)) continue;
    const int64_t t = total_of(x, err);
    tot[q] = t;
    if (stat) stat[n] = (int32_t)(t - (int64_t)(uint32_t)x + img[n]);
  }
  auto stats = [&](uint64_t x, int n, int64_t t) {
    nfeas += 1;
    minidx = min(minidx, n);
    ht += ((int64_t)((x >> 48) & 0xff) == mt);
    ha += ((int64_t)((x >> 32) & 0xffff) == ma);
    tmin = min(tmin, t);
    tmax = max(tmax, t);
  };
#pragma unroll
  for (int q = 0; q < kTopQ; q++) {
    const int n = tid + q * BLOCK;
    if (tot[q] != BIG) stats(rec[n], n, tot[q]);
  }
  for (int n = tid + kTopQ * BLOCK; n < N; n += BLOCK) {
    const uint64_t x = rec[n];
    if (x >> 63) {
      const int64_t t = total_of(x, err);
      stats(x, n, t);
      if (stat) stat[n] = (int32_t)(t - (int64_t)(uint32_t)x + img[n]);
    }
  }
  {
    const int64_t w0 = wave_min64(tmin), w1 = -wave_min64(-tmax);
    const int32_t i0 = wave_sum32(nfeas), i1 = wave_min32(minidx), i2 = wave_sum32(ht), i3 = wave_sum32(ha);
    const uint32_t i4 = wave_or32(err);
    if (lane == 0) {
      s_r[wv][0] = w0;
      s_r[wv][1] = w1;
      s_i[wv][0] = i0;
      s_i[wv][1] = i1;
      s_i[wv][2] = i2;
      s_i[wv][3] = i3;
      s_i[wv][4] = (int32_t)i4;
    }
  }
  __syncthreads();
  int64_t gmin = BIG, gmax = -BIG;
  int32_t gn = 0, gidx = 0x7fffffff, ght = 0, gha = 0, gerr = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    gmin = min(gmin, (int64_t)s_r[i][0]);
    gmax = max(gmax, (int64_t)s_r[i][1]);
    gn += s_i[i][0];
    gidx = min(gidx, s_i[i][1]);
    ght += s_i[i][2];
    gha += s_i[i][3];
    gerr |= s_i[i][4];
  }
  const int K = min(j + 1 + a.k_extra, gn);
  if (tid == 0) {
    P1Stats s;
    s.nfeas = gn;
    s.minidx = gidx;
    s.mt = (int32_t)mt;
    s.ma = (int32_t)ma;
    s.ht = ght;
    s.ha = gha;
    s.err = gerr;
    s.K = K;
    s.inv_mt = mt ? 1.0f / (float)mt : 1.0f;
    s.inv_ma = ma ? 1.0f / (float)ma : 1.0f;
    s.pad = 0;
    if (a.tk_sc) {
#pragma unroll
      for (int w = 0; w < (int)(sizeof(P1Stats) / 4); w++)
        st_sc(reinterpret_cast<int32_t*>(&a.p1[j]) + w, reinterpret_cast<const int32_t*>(&s)[w]);
    } else {
      a.p1[j] = s;
    }
  }
  if (K == 0) return;
  // dense key: larger = better (higher total, then lower node index); distinct per node
  auto dkey = [&](int64_t t, int n) -> int64_t { return (t - gmin) * (int64_t)N + (N - 1 - n); };
  auto each_key = [&](auto&& f) {   // f(dense key, total, node) for every feasible node
#pragma unroll
    for (int q = 0; q < kTopQ; q++) {
      const int n = tid + q * BLOCK;
      if (tot[q] != BIG) f(dkey(tot[q], n), tot[q], n);
    }
    for (int n = tid + kTopQ * BLOCK; n < N; n += BLOCK) {
      const uint64_t x = rec[n];
      uint32_t e = 0;
      if (x >> 63) {
        const int64_t t = total_of(x, e);
        f(dkey(t, n), t, n);
      }
    }
  };
  // Radix select of the K-th largest dense key: 11-bit digits from the top
  // (two levels at configs[1]'s ranges), one LDS histogram per level, the bin
  // holding the K-th key found by one wave's suffix sums.
  constexpr int RB = 11, NB = 1 << RB, PL = NB / 64;
  __shared__ int32_t s_hist[NB];
  __shared__ int32_t s_sel[2];   // selected bin, keys in higher bins
  const int64_t dmax = dkey(gmax, 0);
  const int top_bit = 64 - __builtin_clzll((unsigned long long)dmax | 1ull);
  int64_t prefix = 0;   // the digits fixed so far (dkey >> (shift + RB))
  int need = K;         // keys still to take at or below the prefix
  for (int shift = ((top_bit - 1) / RB) * RB; shift >= 0; shift -= RB) {
    for (int i = tid; i < NB; i += BLOCK) s_hist[i] = 0;
    __syncthreads();
    each_key([&](int64_t d, int64_t, int) {
      if (shift + RB >= 63 || (d >> (shift + RB)) == prefix) atomicAdd(&s_hist[(d >> shift) & (NB - 1)], 1);
    });
    __syncthreads();
    if (wv == 0) {
      int32_t h[PL];
      int32_t sum = 0;
#pragma unroll
      for (int i = 0; i < PL; i++) {
        h[i] = s_hist[lane * PL + i];
        sum += h[i];
      }
      int32_t suf = sum;   // keys in this lane's bins and every higher lane's
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t v = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += v;
      }
      const int32_t above = suf - sum;
      if (above < need && suf >= need) {
        int32_t acc = above, b = lane * PL;
#pragma unroll
        for (int i = PL - 1; i >= 0; i--) {
          if (acc + h[i] >= need) {
            b = lane * PL + i;
            break;
          }
          acc += h[i];
        }
        s_sel[0] = b;
        s_sel[1] = acc;
      }
    }
    __syncthreads();
    prefix = (prefix << RB) | s_sel[0];
    need -= s_sel[1];
  }
  const int64_t thr = prefix;   // the K-th largest dense key: exactly K keys are >= it
  // collect the K keys, then sort them descending by rank (phase 2 takes the
  // first entry outside C): a key's position is the number of larger keys
  __shared__ uint64_t s_keys[KSG_BATCH_MAX];
  each_key([&](int64_t d, int64_t t, int n) {
    if (d >= thr) {
      const int pos = atomicAdd(&s_pos, 1);
      if (pos < KSG_BATCH_MAX) s_keys[pos] = argmax_key(t, n);
    }
  });
  __syncthreads();
  uint64_t* out = a.top + (size_t)j * KSG_BATCH_MAX;
  for (int i = tid; i < K; i += BLOCK) {
    const uint64_t x = s_keys[i];
    int r = 0;
    for (int m = 0; m < K; m++) r += s_keys[m] > x ? 1 : 0;
    if (a.tk_sc) st_sc(out + r, x);
    else out[r] = x;
  }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ksg_batch_topk(BatchArgs a) {
  batch_topk_body<BLOCK>(a);
  if (a.tk_done) {   // hand-off to the walk: every workgroup releases its outputs, the last one signals
    if (a.tk_sc) {   // sc0 sc1 stores: every wave drains them, no release fence
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
      __threadfence();
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      using G1 = __attribute__((address_space(1))) unsigned;
      const unsigned old = __hip_atomic_fetch_add((G1*)a.tk_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x - 1) {
        __hip_atomic_store((G1*)a.tk_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.tk_sc) __hip_atomic_store((G1*)a.tk_done, a.tk_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_store((G1*)a.tk_done, a.tk_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// The slot walk's per-wave partials (ksg_batch_phase2s).
struct WRed {
  uint64_t k0, k1;
  int32_t feas1, live, lost_t, lost_a, cmin, err;
};

// Phase 2, the slot walk (the fallback outside the speculate-and-verify walk's
// scope, and the captured queues).  256 lanes;
// lane i owns changed slot i (the i-th node assumed onto in this batch) and
// keeps that node's phase-1 records in registers, one pod ahead.  Per pod j:
//   X  every lane: spec = the first entry of the sorted top set T_j outside C
//      (ballot over the first 64 entries: the best unchanged node unless all
//      64 are changed); issue pod j+1's loads (records of C, of spec for the
//      next slot's owner, the top set T_{j+1}; wave 0 also spec's columns),
//      all unconditional and unconverted so that nothing waits on them
//      before Y; re-evaluate the lane's changed node on its live slot (one
//      bulk LDS read of the slot, branch-free filter, reciprocal-multiply
//      divisions with an exact correction, Go's float64 BalancedAllocation);
//      DPP reductions; one partial per wave into LDS.
//   -- barrier --
//   Y  every wave folds the four partials and takes the same decision; wave
//      0 assumes the pod into its slot (LDS) and stores the node's new columns
//      (global); the next slot's owner keeps spec's records (or reloads on a
//      miss); the prefetched top set goes to LDS.
//   -- barrier --
// The selected node is either the best unchanged node or a changed one, so
// outside the rare renormalisation every load pod j+1 needs is issued a pod
// early.  RM bounds the resource columns (slot layout fixed at compile time).

// slot row (int64 words): alloc/requested pairs of columns 0..RM-1, then
// nonzero cpu, nonzero memory, pod count, allowed pods, f32 1/alloc of cpu and
// memory (qdiv estimates), f64 alloc of cpu and memory (BalancedAllocation).
template <int RM>
struct SlotLayout {
  static constexpr int NZC = 2 * RM, NZM = 2 * RM + 1, PODS = 2 * RM + 2, ALLOWED = 2 * RM + 3;
  static constexpr int INVC = 2 * RM + 4, INVM = 2 * RM + 5, DAC = 2 * RM + 6, DAM = 2 * RM + 7;
  static constexpr int W = 2 * RM + 8;
  // LDS row stride (int64 words): 2 words of padding put lane i's row 4i banks
  // (mod 64) from lane 0's, so the per-lane 16-byte reads of a row hit disjoint
  // banks instead of all lanes hitting the same bank
  static constexpr int STRIDE = W + 2;
};

struct P2Part {
  uint64_t k0, bu;           // best changed key, best unchanged key (in T_j \ C; only when
                             // the first 64 entries of T_j are all changed)
  uint32_t cnt;              // this wave's feas1 | live << 8 | lost_t << 16 | lost_a << 24 (each <= 64)
  int32_t kidx;              // slot of k0, -1 if not in this wave
};

// qdiv(), ddiv(): ksched_device.h

// CmProf / cm_prof: ksched_device.h

// Per-pod values of the changed-node evaluation, read from LDS in one batch.
template <int RM>
struct PodHot {
  int64_t req[RM];
  int64_t nz_cpu, nz_mem;
  uint32_t req_mask;   // bit r: NodeResourcesFit filter checks column r for this pod
  bool fit_on;         // NodeResourcesFit filter runs for this pod
  int64_t w_fit, w_ba, w_t, w_a;   // weight if the plugin scores this pod, else 0
};

template <int RM>
__device__ __forceinline__ PodHot<RM> pod_hot(const ksg_pod& p, const ksg_profile& prof, bool fit_filter_on, int R) {
  PodHot<RM> h;
  uint32_t m = 0;
#pragma unroll
  for (int r = 0; r < RM; r++) {
    h.req[r] = p.req[r];
    const bool chk = r < R && h.req[r] > 0 && !(r >= 3 && ((prof.fit_ignored_res >> r) & 1u));
    m |= chk ? 1u << r : 0u;
  }
  h.nz_cpu = p.nz_cpu;
  h.nz_mem = p.nz_mem;
  h.req_mask = m;
  h.fit_on = fit_filter_on && !((p.filter_skip >> KSG_PL_NODE_RESOURCES_FIT) & 1u);
  const uint32_t smask = prof.score_mask & ~p.score_skip;
  h.w_fit = (smask & bit(KSG_PL_NODE_RESOURCES_FIT)) ? prof.weight[KSG_PL_NODE_RESOURCES_FIT] : 0;
  h.w_ba = (smask & bit(KSG_PL_BALANCED_ALLOCATION)) ? prof.weight[KSG_PL_BALANCED_ALLOCATION] : 0;
  h.w_t = (smask & bit(KSG_PL_TAINT_TOLERATION)) ? prof.weight[KSG_PL_TAINT_TOLERATION] : 0;
  h.w_a = (smask & bit(KSG_PL_NODE_AFFINITY)) ? prof.weight[KSG_PL_NODE_AFFINITY] : 0;
  return h;
}

// NodeResourcesFit score + BalancedAllocation score of a changed node from its
// slot row w, when both score {cpu, memory}: the results of fit_score /
// ba_score, computed without branches (a column with zero allocatable is left
// out by selects) so that the two chains interleave.
template <int RM>
__device__ __forceinline__ void cm_scores(const CmProf& m, const PodHot<RM>& h, const int64_t (&w)[SlotLayout<RM>::W],
                                          int64_t& fit, int64_t& ba) {
  using SL = SlotLayout<RM>;
  const int64_t ac = w[2 * KSG_RES_CPU], am = w[2 * KSG_RES_MEM];
  const bool hc = ac > 0, hm = am > 0;
  const int64_t sac = hc ? ac : 1, sam = hm ? am : 1;
  const float ic = __int_as_float((int32_t)w[SL::INVC]), im = __int_as_float((int32_t)w[SL::INVM]);
  const int64_t qc = w[SL::NZC] + h.nz_cpu, qm = w[SL::NZM] + h.nz_mem;
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
  const float i_ws = m.inv_ws, i_wc = m.inv_wc, i_wm = m.inv_wm;
  float iws = __builtin_amdgcn_readfirstlane(0) ? 0.0f : i_wm;   // (selects on values, not on
  iws = hc ? i_wc : iws;                                         //  member addresses: no scratch)
  iws = hc && hm ? i_ws : iws;
  fit = ws == 0 ? 0 : qdiv(num, ws, iws);
  const double dac = hc ? __longlong_as_double(w[SL::DAC]) : 1.0, dam = hm ? __longlong_as_double(w[SL::DAM]) : 1.0;
  double fc = ddiv((double)(w[2 * KSG_RES_CPU + 1] + h.req[KSG_RES_CPU]), dac);
  double fm = ddiv((double)(w[2 * KSG_RES_MEM + 1] + h.req[KSG_RES_MEM]), dam);
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = hc && hm ? fabs((fc - fm) / 2) : 0.0;   // |f0 - f1| is symmetric in the column order
  ba = (int32_t)((1 - sd) * (double)100);
}

// cm_scores in 32-bit integers with memory in MiB, for runs whose ranges the
// host and ksg_range32 checked (the N32 instances): the same quotients as the
// int64 form (memory quantities are whole MiB; every product stays below
// 2^30).  The row's INVM / DAC / DAM words hold the N32 decode of
// slot_word_value: 1 / (memory MiB) and ddiv_rcp of cpu and memory MiB.
template <int RM>
__device__ __forceinline__ void cm_scores32(const CmProf& m, const PodHot<RM>& h,
                                            const int64_t (&w)[SlotLayout<RM>::W], int64_t& fit, int64_t& ba) {
  using SL = SlotLayout<RM>;
  const int32_t ac = (int32_t)w[2 * KSG_RES_CPU], am = (int32_t)(w[2 * KSG_RES_MEM] >> 20);
  const bool hc = ac > 0, hm = am > 0;
  const int32_t sac = hc ? ac : 1, sam = hm ? am : 1;
  const float ic = __int_as_float((int32_t)w[SL::INVC]), im = __int_as_float((int32_t)w[SL::INVM]);
  const int32_t qc = (int32_t)w[SL::NZC] + (int32_t)h.nz_cpu;
  const int32_t qm = (int32_t)(w[SL::NZM] >> 20) + (int32_t)(h.nz_mem >> 20);
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
  const int32_t num = (hc ? sc * wc : 0) + (hm ? sm * wm : 0);
  const int32_t ws = (hc ? wc : 0) + (hm ? wm : 0);
  float iws = __builtin_amdgcn_readfirstlane(0) ? 0.0f : m.inv_wm;
  iws = hc ? m.inv_wc : iws;
  iws = hc && hm ? m.inv_ws : iws;
  fit = ws == 0 ? 0 : qdiv32(num, ws, iws);
  const int32_t nc_ = (int32_t)w[2 * KSG_RES_CPU + 1] + (int32_t)h.req[KSG_RES_CPU];
  const int32_t nm_ = (int32_t)(w[2 * KSG_RES_MEM + 1] >> 20) + (int32_t)(h.req[KSG_RES_MEM] >> 20);
  double fc = ddiv_r((double)nc_, (double)sac, __longlong_as_double(w[SL::DAC]));
  double fm = ddiv_r((double)nm_, (double)sam, __longlong_as_double(w[SL::DAM]));
  fc = fc > 1 ? 1 : fc;
  fm = fm > 1 ? 1 : fm;
  const double sd = hc && hm ? fabs((fc - fm) / 2) : 0.0;
  ba = (int32_t)((1 - sd) * (double)100);
}

template <int RM>
__device__ __forceinline__ void slot_row_cols(const int64_t (&w)[SlotLayout<RM>::W], NodeCols& L) {
  using SL = SlotLayout<RM>;
#pragma unroll
  for (int r = 0; r < KSG_MAX_RES; r++) {
    L.alloc[r] = r < RM ? w[2 * (r < RM ? r : 0)] : 0;
    L.req[r] = r < RM ? w[2 * (r < RM ? r : 0) + 1] : 0;
  }
  L.nz_cpu = w[SL::NZC];
  L.nz_mem = w[SL::NZM];
  L.pod_count = (int32_t)w[SL::PODS];
  L.allowed = (int32_t)w[SL::ALLOWED];
}

// Slot word `lane` of node n, loaded without branches (every lane issues the
// same two loads from valid addresses); decode with slot_word_value().
template <int RM>
struct SlotFetch {
  int64_t v64;
  int32_t v32;
};
// The addresses slot_word_fetch selects, reduced once per walk to a lane
// base plus a per-node step (1 or 2 words), so a fetch is one multiply-add
// per pointer instead of the per-lane selects.
struct SlotPlan {
  const int64_t* b64;
  const int32_t* b32;
  int s64, s32;
};
template <int RM, bool N32 = false>
__device__ __forceinline__ SlotPlan slot_plan(const DevCluster& c, const DevState& st, int lane, int R) {
  using SL = SlotLayout<RM>;
  const size_t N = c.N;
  const int r = lane >> 1;
  SlotPlan q{c.alloc, c.allowed, 1, 1};
  if (lane == SL::PODS) q.b32 = st.pod_count;
  if (lane < 2 * RM && r < R) q.b64 = ((lane & 1) ? st.requested : c.alloc) + (size_t)r * N;
  else if (lane == SL::NZC || lane == SL::NZM) q.b64 = st.nonzero + (size_t)(lane - SL::NZC) * N;
  else if (N32 && (lane == SL::DAC || lane == SL::DAM)) {
    q.b64 = reinterpret_cast<const int64_t*>(c.rcp64) + (lane == SL::DAM);
    q.s64 = 2;
  } else if (lane == SL::INVC || lane == SL::DAC) q.b64 = c.alloc + (size_t)KSG_RES_CPU * N;
  else if (lane == SL::INVM || lane == SL::DAM) q.b64 = c.alloc + (size_t)KSG_RES_MEM * N;
  if (N32 && (lane == SL::INVC || lane == SL::INVM)) {
    q.b32 = reinterpret_cast<const int32_t*>(c.rcp32) + (lane == SL::INVM);
    q.s32 = 2;
  }
  return q;
}
template <int RM>
__device__ __forceinline__ SlotFetch<RM> slot_plan_fetch(const SlotPlan& q, int n) {
  return SlotFetch<RM>{q.b64[(size_t)n * q.s64], q.b32[(size_t)n * q.s32]};
}

template <int RM, bool N32 = false>
__device__ __forceinline__ SlotFetch<RM> slot_word_fetch(const DevCluster& c, const DevState& st, int lane, int R,
                                                          int n) {
  using SL = SlotLayout<RM>;
  const size_t N = c.N;
  const int r = lane >> 1;
  const int64_t* p64 = c.alloc + n;   // harmless default
  const int32_t* p32 = lane == SL::PODS ? st.pod_count + n : c.allowed + n;
  if (lane < 2 * RM && r < R) p64 = ((lane & 1) ? st.requested : c.alloc) + (size_t)r * N + n;
  else if (lane == SL::NZC || lane == SL::NZM) p64 = st.nonzero + (size_t)(lane - SL::NZC) * N + n;
  else if (N32 && (lane == SL::DAC || lane == SL::DAM))   // the per-node reciprocals, no decode
    p64 = reinterpret_cast<const int64_t*>(c.rcp64) + 2 * (size_t)n + (lane == SL::DAM);
  else if (lane == SL::INVC || lane == SL::DAC) p64 = c.alloc + (size_t)KSG_RES_CPU * N + n;
  else if (lane == SL::INVM || lane == SL::DAM) p64 = c.alloc + (size_t)KSG_RES_MEM * N + n;
  if (N32 && (lane == SL::INVC || lane == SL::INVM))
    p32 = reinterpret_cast<const int32_t*>(c.rcp32) + 2 * (size_t)n + (lane == SL::INVM);
  return SlotFetch<RM>{*p64, *p32};
}
template <int RM, bool N32 = false>
__device__ __forceinline__ int64_t slot_word_value(const SlotFetch<RM>& f, int lane, int R) {
  using SL = SlotLayout<RM>;
  if (lane == SL::PODS || lane == SL::ALLOWED) return (int64_t)f.v32;
  if (lane < 2 * RM) return (lane >> 1) < R ? f.v64 : 0;
  if (N32) {   // cm_scores32's words: DevCluster::rcp32 / rcp64 as fetched
    if (lane == SL::INVC || lane == SL::INVM) return (int64_t)(uint32_t)f.v32;
    if (lane == SL::DAC || lane == SL::DAM) return f.v64;
  }
  if (lane == SL::INVC || lane == SL::INVM)   // qdiv's estimate: v_rcp_f32 (1 ulp) is within its correction
    return (int64_t)(uint32_t)__float_as_int(f.v64 > 0 ? __builtin_amdgcn_rcpf((float)f.v64) : 1.0f);
  if (lane == SL::DAC || lane == SL::DAM) return __double_as_longlong((double)f.v64);
  return lane < SL::W ? f.v64 : 0;
}

// N32: the run's ranges were checked for cm_scores32 (ksg_range32)
template <int RM, int BLOCK, bool N32 = false>
__global__ __launch_bounds__(BLOCK) void ksg_batch_phase2s(BatchArgs a) {
  using SL = SlotLayout<RM>;
  constexpr int NW = BLOCK / 64, SW = SL::W;
  static_assert(BLOCK % 64 == 0 && BLOCK <= KSG_BATCH_MAX, "one lane per changed slot of a batch of <= BLOCK pods");
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ P1Stats s_p1[KSG_BATCH_MAX];
  __shared__ int32_t s_clist[KSG_BATCH_MAX];
  __shared__ uint64_t s_ce[KSG_BATCH_MAX];     // live record of changed slot i (renormalisation)
  __shared__ P2Part s_part[2][NW];             // by pod parity (one barrier per pod)
  __shared__ WRed s_w[NW];
  __shared__ ksg_result s_res[KSG_BATCH_MAX];  // per-pod results, stored after the walk
  __shared__ uint8_t s_touched[KSG_BATCH_MAX];  // two-batch window: slot assumed onto in this batch

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  const int cm_words = (((N + 31) / 32) + 3) & ~3;
  constexpr int POD_WORDS = sizeof(ksg_pod) / 4;
  uint32_t* s_cmask = reinterpret_cast<uint32_t*>(s_dyn);
  ksg_pod* s_pods = reinterpret_cast<ksg_pod*>(s_dyn + cm_words);
  int32_t* s_prog = s_dyn + cm_words + a.nb * POD_WORDS;
  int64_t* s_slot = reinterpret_cast<int64_t*>(s_dyn + ((cm_words + a.nb * POD_WORDS + a.prog_len + 3) & ~3));

  if (a.tk_done) {   // this batch's top-k (second stream) is done: poll, then acquire
    if (tid == 0) {
      using G1 = __attribute__((address_space(1))) unsigned;
      unsigned spins = 0;
      while (__hip_atomic_load((G1*)a.tk_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.tk_seq) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) {
          __hip_atomic_store((G1*)a.tk_timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  for (int i = tid; i < cm_words; i += BLOCK) s_cmask[i] = 0;
  for (int i = tid; i < a.nb * POD_WORDS; i += BLOCK)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + a.b0)[i];
  for (int i = tid; i < a.prog_len; i += BLOCK) s_prog[i] = a.prog[a.prog_lo + i];
  for (int i = tid; i < a.nb * (int)(sizeof(P1Stats) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(s_p1)[i] = reinterpret_cast<const int32_t*>(a.p1)[i];
  for (int i = tid; i < (int)(sizeof(ksg_profile) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  __syncthreads();
  const CmProf cm = cm_prof(s_prof);
  const bool ipa_filter = ipa_in_filter(s_prof);
  const bool ipa_score = ((s_prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;
  const SlotPlan plan = slot_plan<RM, N32>(c, a.st, lane, R);

  auto changed = [&](int n) { return ((s_cmask[n >> 5] >> (n & 31)) & 1u) != 0; };
  int nc = 0;                  // |C|, block-uniform
  int my_node = 0;             // node of slot tid (tid < nc)
  uint64_t my_rec = 0;         // pod j's phase-1 record at my_node
  int32_t my_img = 0;
  int32_t my_stat = 0;         // N32: pod j's static part of the total at my_node (a.stat)
  // Two-batch window (run_pipe with the slot walk): this batch's phase 1 saw
  // the state before the previous batch's assumes, so the nodes the previous
  // batch touched start as changed slots with their live rows.  Their phase-1
  // records stay usable: an assume only ever removes capacity, so a record
  // that says infeasible stays infeasible, and everything else about the node
  // is re-evaluated on the row (the top sets hold k_extra = |carry| more keys).
  if (a.carry) {
    nc = *a.carry_n;
    for (int t = tid; t < nc * SW; t += BLOCK) {
      const int i = t / SW, w = t - i * SW;
      const SlotFetch<RM> f = slot_word_fetch<RM, N32>(c, a.st, w, R, a.carry[i]);
      s_slot[(size_t)i * SL::STRIDE + w] = slot_word_value<RM, N32>(f, w, R);
    }
    if (tid < nc) {
      my_node = a.carry[tid];
      s_clist[tid] = my_node;
      atomicOr(&s_cmask[my_node >> 5], 1u << (my_node & 31));
      my_rec = a.rec[my_node];
      my_img = a.img[my_node];
      if constexpr (N32) my_stat = a.stat[my_node];
    }
  }
  if (tid < KSG_BATCH_MAX) s_touched[tid] = 0;
  __syncthreads();
  // One barrier per pod.  Every wave keeps the first 64 entries of T_j in its
  // lanes (t64) with their changed flags (t_chg, computed a pod ahead); a
  // slot's row is written only by its owner wave (the wave of lanes that
  // evaluate it), so its next read is in program order; the block-uniform rare
  // paths read the LDS tables after barrier 1, which orders them after every
  // earlier pod's writes.  A wave may still be in pod j - 1's assume while
  // another evaluates pod j: the changed-set reads before barrier 1 add
  // prev_sel, and the per-wave partials alternate by pod parity.
  uint64_t t64 = a.top[lane];
  bool t_chg = lane < s_p1[0].K ? changed(key_node(t64)) : true;
  int prev_sel = -1;
#ifdef KSG_STAMPS
  unsigned long long st_acc[16] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif
  KSG_STAMP(0);
  for (int j = 0; j < a.nb; j++) {
    const ksg_pod& p = s_pods[j];
    const ksg_profile& prof = s_prof;
    const P1Stats s1 = s_p1[j];
    const PodHot<RM> h = pod_hot<RM>(p, prof, fit_filter_on, R);
    // Every LDS read of the pod's setup is issued here, in straight-line code,
    // so they share one round trip (branches on lane or tid would serialise them).
    const int rl = (lane >> 1) < RM ? (lane >> 1) : 0;
    const int64_t req_l = p.req[rl];
    const int32_t p_commit = p.commit, p_ipa = p.ipa;
    const uint32_t p_skip = p.score_skip;
    // this lane's word of the assume (row word `lane` += delta), computed off the critical path
    const int64_t row_delta = lane < 2 * RM ? ((lane & 1) && (lane >> 1) < R ? req_l : 0)
                              : lane == SL::NZC ? h.nz_cpu
                              : lane == SL::NZM ? h.nz_mem
                              : lane == SL::PODS ? 1 : 0;
    const bool has_commit = p_commit >= 0;
    // ipa_skip_bits for an unscored / scored result, without the call's branches
    const bool ipa_none = p_ipa < 0;
    const uint32_t st_pf = ipa_none && ipa_filter ? KSG_ST_IPA_PREFILTER_SKIP : 0u;
    const bool ps_skip = ipa_none && ipa_score && !((p_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u);
    const uint32_t pod_status = st_pf, pod_skip = p_skip;
    const uint32_t pod_status_s = KSG_ST_SCORED | st_pf | (ps_skip ? KSG_ST_IPA_PRESCORE_SKIP : 0u);
    const uint32_t pod_skip_s = p_skip | (ps_skip ? bit(KSG_PL_INTER_POD_AFFINITY) : 0u);
    const int64_t mt1 = s1.mt, ma1 = s1.ma;
    const bool more = j + 1 < a.nb;
    KSG_STAMP(8);
    const int jn = more ? j + 1 : j;   // row of the next-pod loads (always a valid row)

    // ---- X1: speculated best unchanged node (sorted T_j, first 64 entries) --
    // T_j is sorted, so its first entry outside C is the best unchanged key;
    // every wave computes it identically.  Only when all of the first 64
    // entries are changed does the best unchanged key need a block reduction.
    int spec = -1;
    uint64_t bu_key = 0;
    bool bu_full = false;
    {
      const uint64_t m = __ballot(lane < s1.K && !t_chg);
      if (m) {
        bu_key = readlane64(t64, __builtin_ctzll(m));
        spec = key_node(bu_key);
      }
      bu_full = m == 0 && s1.K > 64;
    }
    KSG_STAMP(9);
    // ---- X2: pod j+1's loads (consumed in Y) ----------------------------------
    const int K1 = more ? s_p1[j + 1].K : 0;
    const int nn = tid < nc ? my_node : (spec >= 0 ? spec : 0);
    uint64_t nx_rec = a.rec[(size_t)jn * N + nn];
    int32_t nx_img = a.img[(size_t)jn * N + nn];
    int32_t nx_stat = 0;
    if constexpr (N32) nx_stat = a.stat[(size_t)jn * N + nn];
    const uint64_t nx_t64 = a.top[(size_t)jn * KSG_BATCH_MAX + lane];
    SlotFetch<RM> col = slot_plan_fetch<RM>(plan, spec >= 0 ? spec : 0);
    KSG_STAMP(1);

    // ---- X3: my changed node on its live slot ---------------------------------
    uint32_t cnt = 0;   // feas1 | live << 8 | lost_t << 16 | lost_a << 24
    uint64_t live = 0, my_key = 0;
    if (tid < nc && (my_rec >> 63)) {
      int64_t sw[SW];
      {
        const int4* src = reinterpret_cast<const int4*>(s_slot + (size_t)tid * SL::STRIDE);
#pragma unroll
        for (int k = 0; k < SW / 2; k++) reinterpret_cast<int4*>(sw)[k] = src[k];
      }
      KSG_STAMP(10);
      const uint64_t x = my_rec;
      cnt = 1;
      const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff;
      bool fits = true;
      if (h.fit_on) {
        fits = sw[SL::PODS] + 1 <= sw[SL::ALLOWED];
#pragma unroll
        for (int r = 0; r < RM; r++) fits = fits && (!((h.req_mask >> r) & 1u) || h.req[r] <= sw[2 * r] - sw[2 * r + 1]);
      }
      if (!fits) {
        cnt += (rt == mt1 ? 1u << 16 : 0u) + (ra == ma1 ? 1u << 24 : 0u);
      } else {
        int64_t fs = 0, bs = 0;
        if (cm.fast) {
          if constexpr (N32) cm_scores32<RM>(cm, h, sw, fs, bs);
          else cm_scores<RM>(cm, h, sw, fs, bs);
        } else {
          NodeCols L;
          slot_row_cols<RM>(sw, L);
          fs = fit_score(prof, p, L);
          bs = ba_score(prof, p, L);
        }
        KSG_STAMP(11);
        int64_t part, total;
        if constexpr (N32) {   // range32_candidate: every weighted sum < 2^30
          // the normalised TaintToleration / NodeAffinity terms come with my_stat (top-k)
          const int32_t fb = (int32_t)fs * (int32_t)h.w_fit + (int32_t)bs * (int32_t)h.w_ba;
          part = my_img + fb;
          total = my_stat + fb;
        } else {
          // 100 * rt < 2^15 and 100 * ra < 2^23: qdiv32's range
          const int32_t nt = mt1 != 0 ? 100 - qdiv32(100 * (int32_t)rt, (int32_t)mt1, s1.inv_mt) : 100;
          const int32_t na = ma1 != 0 ? qdiv32(100 * (int32_t)ra, (int32_t)ma1, s1.inv_ma) : (int32_t)ra;
          part = my_img + fs * h.w_fit + bs * h.w_ba;
          total = part + nt * h.w_t + na * h.w_a;
        }
        my_key = argmax_key(total, my_node);
        cnt += 1u << 8;
        live = pack_rec(part, rt, ra);
      }
    }
    KSG_STAMP(12);
    if (tid < nc) s_ce[tid] = live;
    P2Part* part = s_part[j & 1];
    {
      const uint64_t k0 = wreduce(my_key, OpMaxU64{});
      const uint32_t wc = wreduce(cnt, OpAdd32{});
      const uint64_t mk = __ballot(k0 != 0 && my_key == k0);
      uint64_t bu = 0;
      if (bu_full) {   // best unchanged: this wave's slice of T_j (rare)
        uint64_t tk = 0;
        if (tid < s1.K) {   // (T_j from global memory; prev_sel: see above)
          const uint64_t key = a.top[(size_t)j * KSG_BATCH_MAX + tid];
          const int kn = key_node(key);
          if (!changed(kn) && kn != prev_sel) tk = key;
        }
        bu = wreduce(tk, OpMaxU64{});
      }
      if (lane == 0) {
        P2Part o;
        o.k0 = k0;
        o.bu = bu;
        o.cnt = wc;
        o.kidx = mk ? wv * 64 + __builtin_ctzll(mk) : -1;
        part[wv] = o;
      }
    }
    KSG_STAMP(2);
    lds_barrier();   // X2's loads stay in flight into Y (consumed at the assume)

    // ---- Y: decide (every wave, identically) -------------------------------
    uint64_t k0 = 0, bu = bu_key;
    int32_t kidx = -1;
    int feas1 = 0, live_n = 0, lost_t = 0, lost_a = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const P2Part o = part[i];
      if (o.k0 > k0) { k0 = o.k0; kidx = o.kidx; }
      if (bu_full) bu = o.bu > bu ? o.bu : bu;
      feas1 += o.cnt & 0xff;
      live_n += (o.cnt >> 8) & 0xff;
      lost_t += (o.cnt >> 16) & 0xff;
      lost_a += o.cnt >> 24;
    }
    const int unch = s1.nfeas - feas1;   // unchanged feasible nodes
    int nfeas = unch + live_n;
    // a phase-1 maximum whose every holder became infeasible, or a range error:
    // renormalise with the live maxima over all of pod j's records (rare)
    const bool renorm = nfeas >= 2 && (s1.err || (h.w_t && s1.ht - lost_t <= 0) || (h.w_a && s1.ha - lost_a <= 0));
    int selected = -1, idx = -1;   // idx: slot of the selected node if it is in C
    uint32_t status = 0;
    if (renorm) {
      const PodView v = make_view(c, prof, p, s_prog + (p.blob - a.prog_lo), a.prog);
      const uint64_t* rec = a.rec + (size_t)j * N;
      Red r{0, 0, 0, 0x7fffffff};
      for (int pass = 0; pass < 2; pass++) {
        uint64_t best = 0;
        uint32_t err = 0;
        auto visit = [&](uint64_t x, int n) {
          if (!(x >> 63)) return;
          const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
          if (pass == 0) {
            r.nfeas += 1;
            r.max_t = max(r.max_t, rt);
            r.max_a = max(r.max_a, ra);
          } else {
            const uint64_t key = argmax_key(total_score(v, part, rt, ra, r.max_t, r.max_a, err, nullptr, nullptr), n);
            best = key > best ? key : best;
          }
        };
        for (int n = tid; n < N; n += BLOCK)
          if (!changed(n)) visit(rec[n], n);
        if (tid < nc) visit(s_ce[tid], my_node);
        if (pass == 0) {
          WRed o{0, 0, 0, 0, 0, 0, 0, 0};
          o.k0 = (uint64_t)wreduce(r.max_t, OpMax64{});
          o.k1 = (uint64_t)wreduce(r.max_a, OpMax64{});
          o.live = (int32_t)wreduce((uint32_t)r.nfeas, OpAdd32{});
          if (lane == 0) s_w[wv] = o;
          __syncthreads();
          r = Red{0, 0, 0, 0x7fffffff};
#pragma unroll
          for (int i = 0; i < NW; i++) {
            const WRed o2 = s_w[i];
            r.max_t = max(r.max_t, (int64_t)o2.k0);
            r.max_a = max(r.max_a, (int64_t)o2.k1);
            r.nfeas += o2.live;
          }
          __syncthreads();
        } else {
          WRed o{0, 0, 0, 0, 0, 0, 0, 0};
          o.k0 = wreduce(best, OpMaxU64{});
          o.err = (int32_t)wreduce(err, OpOr32{});
          if (lane == 0) s_w[wv] = o;
          __syncthreads();
          uint64_t gb = 0;
          uint32_t ge = 0;
#pragma unroll
          for (int i = 0; i < NW; i++) {
            gb = s_w[i].k0 > gb ? s_w[i].k0 : gb;
            ge |= (uint32_t)s_w[i].err;
          }
          nfeas = r.nfeas;
          status |= KSG_ST_SCORED;
          if (ge) status |= KSG_ST_SCORE_ERROR;
          else selected = key_node(gb);
          if (selected >= 0 && changed(selected)) {
            const uint64_t mk = __ballot(tid < nc && my_node == selected);
            if (mk) s_w[wv].cmin = wv * 64 + __builtin_ctzll(mk);
            else if (lane == 0) s_w[wv].cmin = -1;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NW; i++) idx = max(idx, s_w[i].cmin);
          }
        }
      }
    } else if (nfeas == 1) {
      if (unch == 1) {
        selected = key_node(bu);
      } else {   // the one live changed node (rare): its wave publishes its slot
        const uint64_t mb = __ballot(tid < nc && live != 0);
        if (mb && lane == 0) s_w[0].live = wv * 64 + __builtin_ctzll(mb);
        __syncthreads();
        idx = s_w[0].live;
        selected = s_clist[idx];
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
    KSG_STAMP(3);

    // ---- Y: assume ----------------------------------------------------------
    const bool added = selected >= 0 && idx < 0;
    if (added && selected != spec) {   // speculation missed: dependent loads
      col = slot_plan_fetch<RM>(plan, selected);
      if (tid == nc) {
        nx_rec = a.rec[(size_t)jn * N + selected];
        nx_img = a.img[(size_t)jn * N + selected];
        if constexpr (N32) nx_stat = a.stat[(size_t)jn * N + selected];
      }
    }
    // pod j+1's state into place (waits for X2's loads, before this pod's
    // stores are issued, so the wait never covers a store)
    if (added && tid == nc) my_node = selected;
    if (tid < nc + (added ? 1 : 0)) {
      my_rec = nx_rec;
      my_img = nx_img;
      my_stat = nx_stat;
    }
    // T_{j+1}'s changed flags: this pod's node may not be in the bitmap yet
    t64 = nx_t64;
    t_chg = lane < K1 ? (changed(key_node(t64)) || key_node(t64) == selected) : true;
    KSG_STAMP(6);
    const int64_t col_val = slot_word_value<RM, N32>(col, lane, R);
    KSG_STAMP(7);
    const int slot = added ? nc : idx;
    if (selected >= 0 && wv == (slot >> 6)) {   // the slot's owner wave
      int64_t* row = s_slot + (size_t)slot * SL::STRIDE;
      // the live columns stay in the row; global memory gets them after the walk
      // (an existing row: an LDS add without return, nothing waits on it)
      if (added) {
        if (lane < SW) row[lane] = col_val + row_delta;
      } else if (lane < SW && row_delta != 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(row + lane), (unsigned long long)row_delta);
      }
      if (lane == 0 && has_commit) {   // PodTopologySpread / InterPodAffinity count tables
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
      if (lane == 0 && added) {
        s_cmask[selected >> 5] |= 1u << (selected & 31);
        s_clist[nc] = selected;
      }
      if (lane == 0 && a.carry_out) s_touched[slot] = 1;
    }
    if (tid == 0) {
      const bool sc = (status & KSG_ST_SCORED) != 0;
      ksg_result res;
      res.selected = selected;
      res.n_feasible = nfeas;
      res.status = status | (sc ? pod_status_s : pod_status);
      res.score_skip = sc ? pod_skip_s : pod_skip;
      s_res[j] = res;
    }
    nc += added ? 1 : 0;
    prev_sel = selected;
    KSG_STAMP(4);
  }
  __syncthreads();
  // No store is on the per-pod path: nothing in the walk reads a changed
  // node's columns from global memory (they live in its LDS row), so the rows
  // and the results go out once, here.
  for (int i = tid; i < nc * SW; i += BLOCK) {
    const int slot = i / SW, w = i - slot * SW, node = s_clist[slot];
    const int64_t val = s_slot[(size_t)slot * SL::STRIDE + w];
    if (w < 2 * RM && (w & 1) && (w >> 1) < R) a.st.requested[(size_t)(w >> 1) * N + node] = val;
    else if (w == SL::NZC || w == SL::NZM) a.st.nonzero[(size_t)(w - SL::NZC) * N + node] = val;
    else if (w == SL::PODS) a.st.pod_count[node] = (int32_t)val;
  }
  for (int i = tid; i < a.nb; i += BLOCK) {
    a.placements[a.out0 + i] = s_res[i].selected;
    if (a.results) a.results[a.out0 + i] = s_res[i];
  }
  for (int i = tid; i < 2 * a.nb; i += BLOCK) a.pmax[i] = 0;   // ready for the next batch's phase 1
  if (a.carry_out) {   // the nodes this batch touched, in slot order, for the next batch
    const bool t = tid < nc && s_touched[tid];
    const uint64_t m = __ballot(t);
    if (lane == 0) s_part[0][wv].cnt = (uint32_t)__popcll(m);
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      base += i < wv ? (int)s_part[0][i].cnt : 0;
      total += (int)s_part[0][i].cnt;
    }
    if (t) a.carry_out[base + __popcll(m & ((1ull << lane) - 1))] = s_clist[tid];
    if (tid == 0) *a.carry_out_n = total;
  }
#ifdef KSG_STAMPS
  if (tid == 0 && a.stamps)
    for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], st_acc[i]);
#endif
}

#if !defined(KSG_PART) || defined(KSG_WITH_BATCH)
#include "ksched_n32.h"
#endif
#if !defined(KSG_PART) || defined(KSG_WITH_BATCH)
#include "ksched_phase2v.h"
#endif
#if !defined(KSG_PART) || defined(KSG_WITH_BATCH)
#include "ksched_capture.h"
#endif
#if !defined(KSG_PART) || defined(KSG_WITH_SWEEP)
#include "ksched_sweep.h"
#endif
#if !defined(KSG_PART) || defined(KSG_WITH_CYCLE)
#include "ksched_cycle.h"
#endif

// ---- queue kernel with PodTopologySpread / InterPodAffinity -------------------
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ksg_queue_topo_kernel(QueueArgs a) {
  constexpr int NW = BLOCK / 64;
  constexpr long long BIG = 0x7fffffffffffffffll;
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ __attribute__((aligned(16))) int32_t s_hist[KSG_HIST_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ TopoProg s_g;
  __shared__ TopoShared s_t;
  __shared__ Red s_red[NW];
  __shared__ uint64_t s_best[NW];
  __shared__ uint32_t s_err[NW];
  __shared__ long long s_r64[NW][4];
  __shared__ int s_size[kMaxSoft];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rep = blockIdx.x;
  const DevCluster& c = a.c;
  const int N = c.N;
  int64_t* requested = a.st.requested + rep * a.st.stride_req;
  int64_t* nonzero = a.st.nonzero + rep * a.st.stride_nz;
  int32_t* pod_count = a.st.pod_count + rep * a.st.stride_pc;
  int32_t* cnt = a.st.cnt + rep * a.st.stride_cnt;
  int32_t* tab = a.st.tab + rep * a.st.stride_tab;
  int32_t* tmpl_total = a.st.tmpl_total + rep * a.st.stride_tt;
  int64_t* partial = a.st.partial + rep * a.st.stride_part;
  uint32_t* ports = a.st.ports ? a.st.ports + rep * a.st.stride_ports : nullptr;
  int64_t* sraw = a.st.sraw + rep * a.st.stride_sraw;
  const bool cap = a.cap_fstatus != nullptr && rep == 0;

  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.profiles + rep)[i_];
  __syncthreads();
  const ksg_profile& prof = s_prof;
  bool ipa_in_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_in_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  const bool ipa_in_score = (prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u;

  for (int k = 0; k < a.count; k++) {
    const int pi = a.first + k;
    __syncthreads();
    stage_pod<BLOCK>(a.pods, a.prog, pi, &s_pod, s_blob);
    __syncthreads();
    const ksg_pod& p = s_pod;
    if (tid == 0) {
      const PodView v0 = make_view(c, prof, p, s_blob, a.prog, true);
      parse_topo(p, s_blob, v0.fskip, v0.smask, s_g);
      layout_slots(c, s_g, s_t);
      long long ma = 0, mh = 0, mp = 0;
      for (int i = 0; i < s_g.n_ma; i++) ma += tmpl_total[s_g.m_anti[i]];
      for (int i = 0; i < s_g.n_mh; i++) mh += tmpl_total[s_g.m_hard[i]];
      for (int i = 0; i < s_g.n_mp; i++) mp += tmpl_total[s_g.m_pref[i]];
      s_t.ipa_skip_filter = !s_g.ipa || (ma == 0 && s_g.n_aff == 0 && s_g.n_anti == 0);
      // PreScore Skip unless some term contributes (pref_any added after the pre-pass)
      s_t.ipa_skip_score = !s_g.ipa || !((prof.hard_pod_affinity_weight > 0 && mh > 0) || mp > 0);
      for (int i = 0; i < kMaxHard; i++) { s_t.hard_min[i] = BIG; s_t.hard_dom[i] = 0; }
      for (int i = 0; i < kMaxSoft; i++) {
        s_t.soft_empty[i] = 0; s_t.soft_present[i] = 0; s_t.soft_empty_seen[i] = 0; s_size[i] = 0;
      }
      s_t.n_ignored = 0;
      s_t.aff_total = 0;
      s_t.pref_any = 0;
    }
    __syncthreads();
    const bool ok = s_t.ok;
    for (int i = tid; i < s_t.words; i += BLOCK) s_hist[i] = 0;
    PodView v = make_view(c, prof, p, s_blob, a.prog, true, ports);
    if (s_t.ipa_skip_filter) v.fskip |= bit(KSG_PL_INTER_POD_AFFINITY);
    const TopoProg& g = s_g;
    const TopoCtx tc{&s_g, &s_t, s_hist, cnt, tab};
    __syncthreads();

    // ---- pre-pass: per-domain counts ------------------------------------
    const bool pre = ok && (g.pts_filter || g.pts_score || g.ipa);
    if (pre) {
      long long lmin[kMaxHard], ldom[kMaxHard], lempty[kMaxSoft], laff = 0, lany = 0;
      for (int i = 0; i < kMaxHard; i++) { lmin[i] = BIG; ldom[i] = 0; }
      for (int i = 0; i < kMaxSoft; i++) lempty[i] = 0;
      for (int n = tid; n < N; n += BLOCK) {
        if (g.pts_filter && has_all(c, g.hard, g.n_hard, 7, n)) {
          for (int i = 0; i < g.n_hard; i++) {
            const int32_t* h = g.hard + 7 * i;
            if (!inclusion(c, v, h[5], h[6], n)) continue;
            const Slot& sl = s_t.hard[i];
            const int32_t x = cnt_at(cnt, N, sl.sel, n);
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
          for (int i = 0; i < g.n_soft; i++) {
            const int32_t* sc = g.soft + 6 * i;
            if (sc[5] || !inclusion(c, v, sc[3], sc[4], n)) continue;
            const Slot& sl = s_t.soft[i];
            uint32_t val = lab(c, sl.col, n);
            if (!val) val = 1;   // node.Labels[key] of a missing key is ""
            const int32_t x = cnt_at(cnt, N, sl.sel, n);
            if (sl.unique) {
              if (val == 1) lempty[i] += x;
            } else {
              atomicAdd(&s_hist[sl.hist + val], x);
            }
          }
        }
        if (g.ipa) {
          if (g.n_aff > 0) {
            const int32_t x = cnt_at(cnt, N, g.sel_all, n);
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
            atomicAdd(&s_hist[sl.hist + val], cnt_at(cnt, N, sl.sel, n));
            atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
          }
          for (int i = 0; i < g.n_pref; i++) {
            const Slot& sl = s_t.pref[i];
            const uint32_t val = lab(c, sl.col, n);
            if (!val) continue;
            const int32_t x = cnt_at(cnt, N, sl.sel, n);
            lany |= x > 0;
            if (!sl.unique) {
              atomicAdd(&s_hist[sl.hist + val], x);
              atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
            }
          }
        }
      }
      for (int i = 0; i < g.n_hard; i++) {
        const long long m = wave_min64(lmin[i]), d = wave_sum64(ldom[i]);
        if (lane == 0 && s_t.hard[i].unique) {
          atomicMin((unsigned long long*)&s_t.hard_min[i], (unsigned long long)m);
          atomicAdd(&s_t.hard_dom[i], (int)d);
        }
      }
      for (int i = 0; i < g.n_soft; i++) {
        const long long e = wave_sum64(lempty[i]);
        if (lane == 0 && e) atomicAdd((unsigned long long*)&s_t.soft_empty[i], (unsigned long long)e);
      }
      laff = wave_sum64(laff);
      lany = wave_sum64(lany);
      if (lane == 0) {
        if (laff) atomicAdd((unsigned long long*)&s_t.aff_total, (unsigned long long)laff);
        if (lany) atomicOr(&s_t.pref_any, 1);
      }
      __syncthreads();
      // minimum over present domains of the non-unique hard slots
      for (int i = 0; i < g.n_hard; i++) {
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
      __syncthreads();
      if (tid == 0) {
        for (int i = 0; i < g.n_hard; i++)   // minMatchNum: 0 when fewer domains than minDomains
          if (s_t.hard_dom[i] < g.hard[7 * i + 3]) s_t.hard_min[i] = 0;
        if (s_t.pref_any) s_t.ipa_skip_score = 0;
      }
      __syncthreads();
    }

    uint32_t* cfs = cap ? a.cap_fstatus + (size_t)k * N : nullptr;
    int64_t* craw = cap ? a.cap_raw + (size_t)k * KSG_NPLUGINS * N : nullptr;
    int64_t* cnorm = cap ? a.cap_norm + (size_t)k * KSG_NPLUGINS * N : nullptr;

    // ---- sweep A: filters + node-local raw scores ----------------------------
    Red r{0, 0, 0, 0x7fffffff};
    int lpres[kMaxSoft] = {0, 0, 0, 0}, lseen[kMaxSoft] = {0, 0, 0, 0}, lign = 0;
    for (int n = tid; n < N && ok; n += BLOCK) {
      const NodeEval e = eval_node(c, prof, v, requested, nonzero, pod_count, n, craw, cnorm, &tc);
      if (cap) cfs[n] = e.st;
      if (e.st != 0) {
        partial[n] = -1;
        continue;
      }
      r.nfeas += 1;
      r.minidx = min(r.minidx, n);
      r.max_t = max(r.max_t, e.rt);
      r.max_a = max(r.max_a, e.ra);
      sraw[n] = e.rt;
      sraw[(size_t)N + n] = e.ra;
      partial[n] = e.part;
      if (g.pts_score) {
        if (g.require_all && !has_all(c, g.soft, g.n_soft, 6, n)) {
          lign += 1;
        } else {
          for (int i = 0; i < g.n_soft; i++) {
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
      }
    }
    {
      Red w;
      w.max_t = wave_max64(r.max_t);
      w.max_a = wave_max64(r.max_a);
      w.nfeas = wave_sum32(r.nfeas);
      w.minidx = wave_min32(r.minidx);
      if (lane == 0) s_red[wv] = w;
      if (g.pts_score) {
        for (int i = 0; i < g.n_soft; i++) {
          const int pr = wave_sum32(lpres[i]), se = (int)wave_or32((uint32_t)lseen[i]);
          if (lane == 0) {
            if (pr) atomicAdd(&s_t.soft_present[i], pr);
            if (se) atomicOr(&s_t.soft_empty_seen[i], 1);
          }
        }
        lign = wave_sum32(lign);
        if (lane == 0 && lign) atomicAdd(&s_t.n_ignored, lign);
      }
    }
    __syncthreads();
    Red gr{0, 0, 0, 0x7fffffff};
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const Red w = s_red[i];
      gr.max_t = max(gr.max_t, w.max_t);
      gr.max_a = max(gr.max_a, w.max_a);
      gr.nfeas += w.nfeas;
      gr.minidx = min(gr.minidx, w.minidx);
    }
    const bool scored = gr.nfeas >= 2;
    const bool do_pts = scored && g.pts_score;
    const bool do_ipa = scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
                        !s_t.ipa_skip_score;
    if (do_pts) {
      // topology sizes: distinct domains among feasible, non-ignored nodes
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        int bits = 0;
        for (int wd = tid; wd < (sl.V + 31) / 32; wd += BLOCK) bits += __popc((uint32_t)s_hist[sl.mark + wd]);
        bits = wave_sum32(bits);
        if (lane == 0 && bits) atomicAdd(&s_size[i], bits);
      }
      __syncthreads();
      if (tid == 0)
        for (int i = 0; i < g.n_soft; i++) {
          const Slot& sl = s_t.soft[i];
          int sz;
          if (g.soft[6 * i + 5]) sz = gr.nfeas - s_t.n_ignored;
          else if (sl.unique) sz = s_t.soft_present[i] + s_t.soft_empty_seen[i];
          else sz = s_size[i];
          s_t.soft_w[i] = c.log_table[sz + 2];   // topologyNormalizingWeight = math.Log(size + 2)
        }
      __syncthreads();
    }
    // ---- sweep B: PodTopologySpread / InterPodAffinity raw scores -------------
    long long pmin = BIG, pmax = 0, imin = BIG, imax = -BIG - 1;
    if (do_pts || do_ipa) {
      for (int n = tid; n < N; n += BLOCK) {
        if (partial[n] < 0) continue;
        if (do_pts) {
          const int64_t x = pts_score_node(c, v, tc, n);
          sraw[2 * (size_t)N + n] = x;
          if (x >= 0) { pmin = min(pmin, (long long)x); pmax = max(pmax, (long long)x); }
          if (cap) craw[(size_t)KSG_PL_POD_TOPOLOGY_SPREAD * N + n] = x < 0 ? 0 : x;
        }
        if (do_ipa) {
          const int64_t y = ipa_score_node(c, prof, tc, n);
          sraw[3 * (size_t)N + n] = y;
          imin = min(imin, (long long)y);
          imax = max(imax, (long long)y);
          if (cap) craw[(size_t)KSG_PL_INTER_POD_AFFINITY * N + n] = y;
        }
      }
      pmin = wave_min64(pmin); pmax = wave_max64(pmax); imin = wave_min64(imin); imax = wave_max64(imax);
      if (lane == 0) { s_r64[wv][0] = pmin; s_r64[wv][1] = pmax; s_r64[wv][2] = imin; s_r64[wv][3] = imax; }
      __syncthreads();
      for (int i = 0; i < NW; i++) {
        pmin = min(pmin, s_r64[i][0]); pmax = max(pmax, s_r64[i][1]);
        imin = min(imin, s_r64[i][2]); imax = max(imax, s_r64[i][3]);
      }
    }
    // ---- sweep C: normalise, weight, argmax ------------------------------------
    int selected = -1;
    uint32_t status = 0;
    if (cap && ok && gr.nfeas == 1 && tid == 0)   // one feasible node: no Score runs, nothing recorded
      for (int q = 0; q < KSG_NPLUGINS; q++) craw[(size_t)q * N + gr.minidx] = cnorm[(size_t)q * N + gr.minidx] = 0;
    if (!ok) {
      status |= KSG_ST_SCORE_ERROR;
    } else if (gr.nfeas == 1) {
      selected = gr.minidx;
    } else if (scored) {
      status |= KSG_ST_SCORED;
      uint64_t best = 0;
      uint32_t err = 0;
      int64_t* ctot = cap ? a.cap_total + (size_t)k * N : nullptr;
      const int64_t w_pts = prof.weight[KSG_PL_POD_TOPOLOGY_SPREAD], w_ipa = prof.weight[KSG_PL_INTER_POD_AFFINITY];
      for (int n = tid; n < N; n += BLOCK) {
        const int64_t part = partial[n];
        if (part < 0) continue;
        int64_t nt = 0, na = 0;
        int64_t total = total_score(v, part, sraw[n], sraw[(size_t)N + n], gr.max_t, gr.max_a, err, &nt, &na);
        if (cap) {
          if (v.smask & bit(KSG_PL_TAINT_TOLERATION)) cnorm[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = nt;
          if (v.smask & bit(KSG_PL_NODE_AFFINITY)) cnorm[(size_t)KSG_PL_NODE_AFFINITY * N + n] = na;
        }
        if (do_pts) {   // PodTopologySpread.NormalizeScore
          const int64_t x = sraw[2 * (size_t)N + n];
          int64_t s;
          if (x < 0) s = 0;
          else if (pmax == 0) s = 100;
          else s = div_small(100 * (pmax + pmin - x), pmax);
          err |= (s < 0 || s > 100);
          total += s * w_pts;
          if (cap) cnorm[(size_t)KSG_PL_POD_TOPOLOGY_SPREAD * N + n] = s;
        }
        if (do_ipa) {   // InterPodAffinity.NormalizeScore (float64 min-max)
          const int64_t y = sraw[3 * (size_t)N + n];
          const int64_t diff = imax - imin;
          double f = 0;
          if (diff > 0) f = (double)100 * ((double)(y - imin) / (double)diff);
          const int64_t s = (int64_t)f;
          err |= (s < 0 || s > 100);
          total += s * w_ipa;
          if (cap) cnorm[(size_t)KSG_PL_INTER_POD_AFFINITY * N + n] = s;
        }
        if (cap) ctot[n] = total;
        const uint64_t key = argmax_key(total, n);
        best = key > best ? key : best;
      }
      best = wave_max_u64(best);
      err = wave_or32(err);
      if (lane == 0) { s_best[wv] = best; s_err[wv] = err; }
      __syncthreads();
      uint64_t gb = 0;
      uint32_t ge = 0;
#pragma unroll
      for (int i = 0; i < NW; i++) {
        gb = s_best[i] > gb ? s_best[i] : gb;
        ge |= s_err[i];
      }
      if (ge) status |= KSG_ST_SCORE_ERROR;
      else selected = key_node(gb);
    }
    uint32_t score_skip = p.score_skip;
    if (ipa_in_filter && s_t.ipa_skip_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
    if (scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) && s_t.ipa_skip_score) {
      status |= KSG_ST_IPA_PRESCORE_SKIP;
      score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
    }
    if (tid == 0) {
      if (a.do_commit && selected >= 0)
        commit_node(c, requested, nonzero, pod_count, cnt, tab, tmpl_total, p,
                    v.commit >= 0 ? s_blob + v.commit : nullptr, selected, 1, ports,
                    v.ports >= 0 ? s_blob + v.ports : nullptr);
      a.placements[(size_t)rep * a.count + k] = selected;
      if (a.results) {
        ksg_result res;
        res.selected = selected;
        res.n_feasible = gr.nfeas;
        res.status = status;
        res.score_skip = score_skip;
        a.results[(size_t)rep * a.count + k] = res;
      }
    }
  }
}

#if !defined(KSG_PART) || defined(KSG_WITH_TOPO)
#include "ksched_topo_tables.h"
#endif
#if !defined(KSG_PART) || defined(KSG_WITH_TOPO)
#include "ksched_topo_win.h"
#include "ksched_topo_coop.h"
#endif

// dst[r * stride + i] = src[i] for every replica r = blockIdx.y (replica state
// initialisation: one launch per array instead of one copy per replica).
template <typename T>
__global__ __launch_bounds__(256) void ksg_broadcast(const T* __restrict__ src, T* __restrict__ dst, size_t len,
                                                     size_t stride) {
  T* d = dst + (size_t)blockIdx.y * stride;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < len; i += (size_t)gridDim.x * 256) d[i] = src[i];
}

// Per replica: Σ requested cpu and Σ requested memory over the nodes (summaries).
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_replica_sums(const int64_t* requested, size_t stride, int N,
                                                        int64_t* out) {
  __shared__ int64_t s_p[2][4];
  const int64_t* q = requested + (size_t)blockIdx.x * stride;
  int64_t a = 0, b = 0;
  for (int n = threadIdx.x; n < N; n += 256) {
    a += q[n];
    b += q[(size_t)N + n];
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

#ifndef KSG_PART
// tables (the per-cycle domain tables, ksg_eval of topology pods): the
// assume's effect on them as lag_apply adds it, for sign +1 (assume) and -1
// (a victim's deletion), from the selectors' counts before the update.
// ksg_commit_kernel's assume with the pod's record and commit program passed
// by value from the host copies (ksg_commit / ksg_uncommit when they fit):
// no dependent loads of the record and program in front of the updates.
constexpr int kCommitSel = 48, kCommitTmpl = 24;
struct CommitArgs {
  int32_t node, sign, ns, nt;
  int64_t req[KSG_MAX_RES];
  int64_t nz_cpu, nz_mem;
  const int32_t* ports;        // the pod's ports program (device pool), or null
  int32_t sel[kCommitSel];
  int32_t tm[kCommitTmpl], tw[kCommitTmpl];
};
__global__ __launch_bounds__(64) void ksg_commit_args_kernel(DevCluster c, DevState st, CommitArgs a, TopoTables t,
                                                             int tables) {
  const int lane = threadIdx.x, N = c.N, node = a.node, sign = a.sign;
  if (lane == 0 && a.ports && st.ports) ports_commit(st.ports, N, node, a.ports, sign);
  if (lane < c.R) st.requested[(size_t)lane * N + node] += sign * a.req[lane];
  if (lane == KSG_MAX_RES) st.nonzero[node] += sign * a.nz_cpu;
  if (lane == KSG_MAX_RES + 1) st.nonzero[(size_t)N + node] += sign * a.nz_mem;
  if (lane == KSG_MAX_RES + 2) st.pod_count[node] += sign;
  if (lane < a.ns) {
    const int sel = a.sel[lane];
    const int old = atomicAdd(st.cnt + (size_t)sel * N + node, sign);
    if (tables) {
      for (int k = t.sp_off[sel]; k < t.sp_off[sel + 1]; k++) {
        const uint32_t v = c.label_val[(size_t)t.sp[2 * k] * N + node];
        if (v) atomicAdd(t.dom + t.sp[2 * k + 1] + v, sign);
      }
      atomicAdd(t.tot + sel, sign);
      const int co = t.cc_off[sel];
      if (co >= 0) {
        const int k = old + sign;
        if (old >= t.Kc - 1 || k < 0 || k >= t.Kc - 1) {
          *t.invalid = 1u;
        } else {
          atomicSub(t.cc + co + old, 1);
          atomicAdd(t.cc + co + k, 1);
        }
      }
    }
  }
  if (lane < a.nt) {
    const int tm = a.tm[lane];
    const uint32_t val = c.label_val[(size_t)c.tmpl_col[tm] * N + node];
    if (val) {
      atomicAdd(st.tab + c.tmpl_off[tm] + val, sign * (c.tmpl_kind[tm] == KSG_TMPL_PREF ? a.tw[lane] : 1));
      atomicAdd(st.tmpl_total + tm, sign);
    }
  }
}

__global__ __launch_bounds__(64) void ksg_commit_kernel(DevCluster c, DevState st, const ksg_pod* pods,
                                                        const int32_t* prog, int pod, int node, int sign,
                                                        TopoTables t, int tables) {
  // commit_node's updates spread over the wave: the node's columns over lanes
  // 0 .. R + 2, one lane per matched selector (its count and, with the
  // tables, its domain / total / count-of-counts entries), one per template;
  // atomics, so a program naming an entry twice adds twice as the serial
  // form does.  (Round 5: one lane walked it all, 4-7 us of dependent loads.)
  const int lane = threadIdx.x;
  if (blockIdx.x != 0) return;
  const ksg_pod& p = pods[pod];
  const int N = c.N;
  if (lane == 0 && p.ports >= 0 && st.ports) ports_commit(st.ports, N, node, prog + p.ports, sign);
  if (lane < c.R) st.requested[(size_t)lane * N + node] += sign * p.req[lane];
  if (lane == KSG_MAX_RES) st.nonzero[node] += sign * p.nz_cpu;
  if (lane == KSG_MAX_RES + 1) st.nonzero[(size_t)N + node] += sign * p.nz_mem;
  if (lane == KSG_MAX_RES + 2) st.pod_count[node] += sign;
  if (p.commit < 0) return;
  const int32_t* cw = prog + p.commit;
  const int ns = cw[0];
  for (int i = lane; i < ns; i += 64) {
    const int sel = cw[1 + i];
    const int old = atomicAdd(st.cnt + (size_t)sel * N + node, sign);
    if (!tables) continue;
    for (int k = t.sp_off[sel]; k < t.sp_off[sel + 1]; k++) {
      const uint32_t v = c.label_val[(size_t)t.sp[2 * k] * N + node];
      if (v) atomicAdd(t.dom + t.sp[2 * k + 1] + v, sign);
    }
    atomicAdd(t.tot + sel, sign);
    const int co = t.cc_off[sel];
    if (co >= 0) {
      const int k = old + sign;   // the node's count after the update
      if (old >= t.Kc - 1 || k < 0 || k >= t.Kc - 1) {
        *t.invalid = 1u;
      } else {
        atomicSub(t.cc + co + old, 1);
        atomicAdd(t.cc + co + k, 1);
      }
    }
  }
  const int32_t* w = cw + 1 + ns;
  const int nt = w[0];
  for (int i = lane; i < nt; i += 64) {
    const int tm = w[1 + 2 * i];
    const uint32_t val = c.label_val[(size_t)c.tmpl_col[tm] * N + node];
    if (!val) continue;
    atomicAdd(st.tab + c.tmpl_off[tm] + val, sign * (c.tmpl_kind[tm] == KSG_TMPL_PREF ? w[2 + 2 * i] : 1));
    atomicAdd(st.tmpl_total + tm, sign);
  }
}
#endif  // KSG_PART

// ksg_commit_batch: commit_node of many (pod, node) pairs, one lane each;
// every column update is an atomic add (or, for the UsedPorts bitmap, an
// atomic or), so lanes sharing a node need no order.
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_commit_batch_kernel(DevCluster c, DevState st, const ksg_pod* pods,
                                                               const int32_t* prog, const int32_t* bp,
                                                               const int32_t* bn, int n_binds) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n_binds) return;
  const ksg_pod& p = pods[bp[k]];
  const int n = bn[k], N = c.N;
  auto add64 = [](int64_t* a, int64_t v) {
    if (v) atomicAdd(reinterpret_cast<unsigned long long*>(a), (unsigned long long)v);
  };
  for (int r = 0; r < c.R; r++) add64(st.requested + (size_t)r * N + n, p.req[r]);
  add64(st.nonzero + n, p.nz_cpu);
  add64(st.nonzero + (size_t)N + n, p.nz_mem);
  atomicAdd(st.pod_count + n, 1);
  if (p.ports >= 0 && st.ports) {
    const int32_t* w = prog + p.ports;
    const int32_t* own = w + 1 + w[0];
    for (int i = 0; i < own[0]; i++) {
      const uint32_t id = (uint32_t)own[1 + i];
      atomicOr(st.ports + (size_t)(id >> 5) * N + n, 1u << (id & 31));
    }
  }
  if (p.commit >= 0) {
    const int32_t* w = prog + p.commit;
    const int ns = *w++;
    for (int i = 0; i < ns; i++) atomicAdd(st.cnt + (size_t)w[i] * N + n, 1);
    w += ns;
    const int nt = *w++;
    for (int i = 0; i < nt; i++) {
      const int t = w[2 * i];
      const uint32_t val = c.label_val[(size_t)c.tmpl_col[t] * N + n];
      if (!val) continue;
      atomicAdd(st.tab + c.tmpl_off[t] + val, c.tmpl_kind[t] == KSG_TMPL_PREF ? w[2 * i + 1] : 1);
      atomicAdd(st.tmpl_total + t, 1);
    }
  }
}
#endif  // KSG_PART

// DefaultPreemption dry run (SelectVictimsOnNode), one lane per candidate
// node: the lane takes the node's live columns, removes every potential
// victim, checks NodeResourcesFit for the preemptor, then reprieves the
// victims most important first.  Only the Fit columns change, so a lane
// works in registers on one NodeCols; victims of a node are few, and the
// pass is off the per-pod critical path (it runs for pods with no feasible
// node only).
#ifndef KSG_PART
// NodePorts in the preemption dry run: which of the preemptor's conflict ids
// (ksg_pod.ports, at most kPreMaxConf: the host refuses more) are set in the
// node's UsedPorts, as a bit mask.  A victim's removal clears the ids it owns
// and its re-addition sets them (set semantics, as ports_commit and upstream
// HostPortInfo: a removal drops an entry another pod on the node may share).
constexpr int kPreMaxConf = 64;
struct PrePorts {
  const int32_t* conf = nullptr;
  int nconf = 0;
  uint64_t bits = 0;
  __device__ void init(const int32_t* w, const uint32_t* used, int N, int n) {
    if (!w || !used) return;
    nconf = w[0] < kPreMaxConf ? w[0] : kPreMaxConf;
    conf = w + 1;
    for (int j = 0; j < nconf; j++) {
      const uint32_t id = (uint32_t)conf[j];
      if ((used[(size_t)(id >> 5) * N + n] >> (id & 31)) & 1u) bits |= 1ull << j;
    }
  }
  __device__ void move(const int32_t* w, int sign) {   // the pod's own ids (w: its ports program)
    if (!conf || !w) return;
    const int32_t* own = w + 1 + w[0];
    for (int i = 0; i < own[0]; i++)
      for (int j = 0; j < nconf; j++)
        if (conf[j] == own[1 + i]) bits = sign > 0 ? bits | (1ull << j) : bits & ~(1ull << j);
  }
  __device__ bool ok() const { return bits == 0; }
};

__global__ __launch_bounds__(256) void ksg_preempt_kernel(DevCluster c, DevState st, const ksg_pod* pods,
                                                          const int32_t* prog, int pod, uint32_t ignored, int fit_on,
                                                          int ports_on, const int32_t* cand, int n_cand,
                                                          const int32_t* off, const int32_t* vic, int32_t* fits,
                                                          uint8_t* victim) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_cand) return;
  const int n = cand[k];
  NodeCols L;
  load_cols(c, st.requested, st.nonzero, st.pod_count, n, L);
  const ksg_pod& p = pods[pod];
  PrePorts pp;
  pp.init(ports_on ? prog + p.ports : nullptr, st.ports, c.N, n);
  const int b = off[k], e = off[k + 1];
  auto move = [&](const ksg_pod& v, int sign) {
#pragma unroll
    for (int r = 0; r < KSG_MAX_RES; r++)
      if (r < c.R) L.req[r] += sign * v.req[r];
    L.nz_cpu += sign * v.nz_cpu;
    L.nz_mem += sign * v.nz_mem;
    L.pod_count += sign;
    pp.move(v.ports >= 0 ? prog + v.ports : nullptr, sign);
  };
  auto passes = [&]() { return pp.ok() && (!fit_on || fit_filter(c, p, L, ignored) == 0); };
  for (int i = b; i < e; i++) move(pods[vic[i]], -1);
  const bool ok = passes();
  fits[k] = ok ? 1 : 0;
  for (int i = b; i < e; i++) {
    uint8_t out = 0;
    if (ok) {
      move(pods[vic[i]], +1);
      if (!passes()) {
        move(pods[vic[i]], -1);
        out = 1;
      }
    }
    victim[i] = out;
  }
}
#endif  // KSG_PART

#if !defined(KSG_PART) || defined(KSG_WITH_PREEMPT)
#include "ksched_preempt.h"
#endif

// DevCluster::rcp32 / rcp64 from the allocatable (static: once per load).
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_node_rcp(DevCluster c, float2* r32, double2* r64) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= c.N) return;
  const int64_t ac = c.alloc[(size_t)KSG_RES_CPU * c.N + n], am = c.alloc[(size_t)KSG_RES_MEM * c.N + n] >> 20;
  const int64_t sc = ac > 0 ? ac : 1, sm = am > 0 ? am : 1;
  r32[n] = float2{__builtin_amdgcn_rcpf((float)sc), __builtin_amdgcn_rcpf((float)sm)};
  r64[n] = double2{ddiv_rcp((double)sc), ddiv_rcp((double)sm)};
}
#endif  // KSG_PART

// Node half of the N32 check (range32_candidate): every value cm_scores32
// will see for any pod of the run stays inside its 32-bit range; the requested
// sums are bounded by max(current, allocatable) (the Fit filter) and the
// non-zero sums by current + allocatable + (placeable pods + 1) x the pods'
// non-zero excess.  Any failure sets *bad (the int64 instances run).
//
// mw = 1: the wide-memory instance (memory in int64 bytes): the cpu half as
// above; memory needs no alignment, only every quantity and reachable sum
// below 2^46, so x 100 stays exact in float64 and below qdiv's 2^53.
#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_range32(DevCluster c, DevState st, int64_t xc, int64_t xm, int32_t count,
                                                   int32_t mw, unsigned* bad) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int N = c.N;
  if (n >= N) return;
  const size_t NN = N;
  constexpr int64_t kMiB = (int64_t)1 << 20, k30 = (int64_t)1 << 30, k31 = ((int64_t)1 << 31) - 1,
                    k46 = (int64_t)1 << 46;
  const int64_t ac = c.alloc[KSG_RES_CPU * NN + n], am = c.alloc[KSG_RES_MEM * NN + n];
  const int64_t rc = st.requested[KSG_RES_CPU * NN + n], rm = st.requested[KSG_RES_MEM * NN + n];
  const int64_t zc = st.nonzero[n], zm = st.nonzero[NN + n];
  const int64_t places = (int64_t)max(0, min(count, c.allowed[n] - st.pod_count[n])) + 1;
  bool ok = ac >= 0 && am >= 0 && rc >= 0 && rm >= 0 && zc >= 0 && zm >= 0;
  ok = ok && ac * 100 < k30 && rc <= k31 && zc + ac + places * xc <= k31;
  if (mw) {
    ok = ok && am < k46 && rm < k46 && zm < k46 && (double)zm + (double)am + (double)places * (double)xm < (double)k46;
  } else {
    ok = ok && ((am | rm | zm) & (kMiB - 1)) == 0;
    ok = ok && (am >> 20) * 100 < k30 && (rm >> 20) <= k31 && (zm >> 20) + (am >> 20) + places * xm <= k31;
  }
  if (!ok) atomicOr(bad, 1u);
}
#endif  // KSG_PART

}  // namespace ksk

#ifndef KSG_PART
#include "ksched_json.h"   // the device annotation serialiser (host TU only)
#endif
