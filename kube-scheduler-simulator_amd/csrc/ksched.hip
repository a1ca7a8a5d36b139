// libksched.so — MI355X (gfx950) Filter/Score evaluator behind the C ABI of
// include/ksched.h.
//
// Kernel structure:
//   ksg_queue_kernel<BLOCK>: one workgroup per scheduling replica, persistent
//   over the pod queue.  Per pod:
//     stage   pod record + its program blob -> LDS (one coalesced copy)
//     sweep A every lane walks nodes n = tid, tid+BLOCK, ...: Filter plugins in
//             profile order with first-rejection exit (RunFilterPlugins), then
//             raw scores; un-normalised plugins (Fit, BalancedAllocation,
//             ImageLocality) are weighted into a partial total on the spot;
//             normalised plugins (TaintToleration, NodeAffinity) keep their raw
//             score and feed block-wide max reductions
//     reduce  wave shuffles + one LDS round: feasible count, first feasible
//             node, per-plugin maxima
//     sweep B (>= 2 feasible nodes) DefaultNormalizeScore, weighted sum,
//             packed (total << 32 | ~node) argmax = selectHost with the
//             lowest-index tie-break
//     assume  one lane commits the pod into the selected node's columns
//   A replica never talks to another workgroup, so there is no inter-workgroup
//   synchronisation at all (the per-pod dependency is inside one CU).
//   ksg_commit_kernel: NodeInfo.AddPod for ksg_commit().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ksched_device.h"

namespace {

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

constexpr uint32_t bit(int p) { return 1u << p; }

__device__ __forceinline__ int64_t wave_max64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t w = __shfl_xor(v, o, 64);
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
      const uint32_t v = c.label_val[(size_t)col * N + n];
      if (!v) continue;
      tab[c.tmpl_off[t] + v] += c.tmpl_kind[t] == KSG_TMPL_PREF ? c.tmpl_weight[t] : 1;
      tmpl_total[t] += 1;
    }
  }
}

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
  const bool cap = a.cap_fstatus != nullptr && rep == 0;

  if (tid < (int)(sizeof(ksg_profile) / 4))
    reinterpret_cast<int32_t*>(&s_prof)[tid] = reinterpret_cast<const int32_t*>(a.profiles + rep)[tid];

  for (int k = 0; k < a.count; k++) {
    const int pi = a.first + k;
    __syncthreads();  // previous pod fully consumed; its commit is visible
    if (tid < (int)(sizeof(ksg_pod) / 4))
      reinterpret_cast<int32_t*>(&s_pod)[tid] = reinterpret_cast<const int32_t*>(a.pods + pi)[tid];
    {
      const int boff = a.pods[pi].blob, blen = a.pods[pi].blob_len;
      for (int i = tid; i < blen; i += BLOCK) s_blob[i] = a.prog[boff + i];
    }
    __syncthreads();
    const ksg_pod& p = s_pod;
    const ksg_profile& prof = s_prof;
    const int boff = p.blob;
    auto rb = [boff](int off) { return off < 0 ? -1 : off - boff; };
    const int32_t* P = s_blob;
    const int tol = rb(p.tol), na_req = rb(p.na_req), na_pref = rb(p.na_pref), img = rb(p.img);
    const int32_t* tolf = P + tol;
    const int32_t* tolp = P + tol + c.W;
    const bool reject = (p.flags & KSG_POD_PREFILTER_REJECT) != 0;
    const uint32_t fskip = p.filter_skip | bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD);
    const uint32_t smask = prof.score_mask & ~p.score_skip &
                           ~(bit(KSG_PL_INTER_POD_AFFINITY) | bit(KSG_PL_POD_TOPOLOGY_SPREAD));
    const int64_t w_fit = prof.weight[KSG_PL_NODE_RESOURCES_FIT];
    const int64_t w_ba = prof.weight[KSG_PL_BALANCED_ALLOCATION];
    const int64_t w_img = prof.weight[KSG_PL_IMAGE_LOCALITY];
    const int64_t w_t = prof.weight[KSG_PL_TAINT_TOLERATION];
    const int64_t w_a = prof.weight[KSG_PL_NODE_AFFINITY];
    uint32_t* cfs = cap ? a.cap_fstatus + (size_t)k * N : nullptr;
    int64_t* craw = cap ? a.cap_raw + (size_t)k * KSG_NPLUGINS * N : nullptr;
    int64_t* cnorm = cap ? a.cap_norm + (size_t)k * KSG_NPLUGINS * N : nullptr;

    // ---- sweep A: filters + raw scores ------------------------------------
    Red r{0, 0, 0, 0x7fffffff};
    for (int n = tid; n < N; n += BLOCK) {
      uint32_t st = 0;
      if (reject || (p.node_set >= 0 && !((((uint32_t)a.prog[p.node_set + (n >> 5)]) >> (n & 31)) & 1u))) {
        st = KSG_FS_NOT_EVALUATED;
      } else {
        for (int kf = 0; kf < prof.n_filter && !st; kf++) {
          const int pl = prof.filter_order[kf];
          if ((fskip >> pl) & 1u) continue;
          switch (pl) {
            case KSG_PL_NODE_UNSCHEDULABLE:
              if (c.unsched[n] && !(p.flags & KSG_POD_TOL_UNSCHED)) st = pl + 1;
              break;
            case KSG_PL_NODE_NAME:
              if (p.node_name != -1 && p.node_name != n) st = pl + 1;
              break;
            case KSG_PL_TAINT_TOLERATION: {
              const int s = untolerated_slot(c, tolf, n);
              if (s >= 0) st = (uint32_t)(pl + 1) | ((uint32_t)s << 8);
              break;
            }
            case KSG_PL_NODE_AFFINITY:
              if (!na_required_match(c, P, na_req, n)) st = (uint32_t)(pl + 1) | (1u << 8);
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
      if (cap) cfs[n] = st;
      if (st == 0) {
        r.nfeas += 1;
        r.minidx = min(r.minidx, n);
        int64_t part = 0;
        if (smask & bit(KSG_PL_NODE_RESOURCES_FIT)) {
          const int64_t s = fit_score(c, prof, p, requested, nonzero, n);
          part += s * w_fit;
          if (cap) { craw[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; cnorm[(size_t)KSG_PL_NODE_RESOURCES_FIT * N + n] = s; }
        }
        if (smask & bit(KSG_PL_BALANCED_ALLOCATION)) {
          const int64_t s = ba_score(c, prof, p, requested, nonzero, n);
          part += s * w_ba;
          if (cap) { craw[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; cnorm[(size_t)KSG_PL_BALANCED_ALLOCATION * N + n] = s; }
        }
        if (smask & bit(KSG_PL_IMAGE_LOCALITY)) {
          const int64_t s = image_score(c, P, img, p.n_containers, n);
          part += s * w_img;
          if (cap) { craw[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; cnorm[(size_t)KSG_PL_IMAGE_LOCALITY * N + n] = s; }
        }
        if (smask & bit(KSG_PL_TAINT_TOLERATION)) {
          const int64_t s = taint_score(c, tolp, n);
          sraw[n] = s;
          r.max_t = max(r.max_t, s);
          if (cap) craw[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = s;
        }
        if (smask & bit(KSG_PL_NODE_AFFINITY)) {
          const int64_t s = na_pref_score(c, P, na_pref, n);
          sraw[(size_t)N + n] = s;
          r.max_a = max(r.max_a, s);
          if (cap) craw[(size_t)KSG_PL_NODE_AFFINITY * N + n] = s;
        }
        partial[n] = part;
      } else {
        partial[n] = -1;
      }
    }
    // ---- reduce ------------------------------------------------------------
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
        int64_t total = part;
        if (smask & bit(KSG_PL_TAINT_TOLERATION)) {
          const int64_t s = sraw[n];
          int64_t v = 100;
          if (g.max_t != 0) v = 100 - 100 * s / g.max_t;
          err |= (v < 0 || v > 100);
          total += v * w_t;
          if (cap) cnorm[(size_t)KSG_PL_TAINT_TOLERATION * N + n] = v;
        }
        if (smask & bit(KSG_PL_NODE_AFFINITY)) {
          const int64_t s = sraw[(size_t)N + n];
          int64_t v = s;
          if (g.max_a != 0) v = 100 * s / g.max_a;
          err |= (v < 0 || v > 100);
          total += v * w_a;
          if (cap) cnorm[(size_t)KSG_PL_NODE_AFFINITY * N + n] = v;
        }
        if (cap) ctot[n] = total;
        const uint64_t key = ((uint64_t)total << 32) | (uint64_t)(0xffffffffu - (uint32_t)n);
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
      else selected = (int)(0xffffffffu - (uint32_t)(gb & 0xffffffffu));
    }
    if (tid == 0) {
      if (a.do_commit && selected >= 0) {
        const int32_t* cp = p.commit >= 0 ? P + rb(p.commit) : nullptr;
        commit_node(c, requested, nonzero, pod_count, cnt, tab, tmpl_total, p, cp, selected);
      }
      a.placements[(size_t)rep * a.count + k] = selected;
      if (a.results) {
        ksg_result res;
        res.selected = selected;
        res.n_feasible = g.nfeas;
        res.status = status;
        res.score_skip = p.score_skip;
        a.results[(size_t)rep * a.count + k] = res;
      }
    }
  }
}

__global__ void ksg_commit_kernel(DevCluster c, DevState st, const ksg_pod* pods, const int32_t* prog, int pod,
                                  int node) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ksg_pod& p = pods[pod];
  commit_node(c, st.requested, st.nonzero, st.pod_count, st.cnt, st.tab, st.tmpl_total, p,
              p.commit >= 0 ? prog + p.commit : nullptr, node);
}

}  // namespace

// ============================================================================
// Host side
// ============================================================================
struct ksg_ctx {
  int device = 0;
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_ms = 0;
  ksg_profile prof{};
  bool have_prof = false, have_nodes = false, have_wl = false;
  // cluster
  DevCluster c{};
  std::vector<void*> allocs;
  int32_t n_pods = 0;
  ksg_pod* d_pods = nullptr;
  int32_t* d_prog = nullptr;
  std::vector<ksg_pod> h_pods;
  int32_t max_blob = 0;
  bool any_topology = false;
  // state (replica 0 = the ctx's own state)
  DevState st{};
  size_t tab_words = 0;
  // load-time snapshot for ksg_reset_state
  int64_t* d_req0 = nullptr;
  int64_t* d_nz0 = nullptr;
  int32_t* d_pc0 = nullptr;
  void* wl_allocs[2] = {nullptr, nullptr};
};

namespace {

int fail(ksg_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

#define HIPC(ctx, expr)                                                                     \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(ctx, KSG_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));    \
  } while (0)

template <typename T>
int dalloc(ksg_ctx* ctx, T** p, size_t count) {
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  hipError_t e = hipMalloc((void**)p, bytes);
  if (e != hipSuccess) return fail(ctx, KSG_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  ctx->allocs.push_back(*p);
  return KSG_OK;
}

template <typename T>
int upload(ksg_ctx* ctx, T** p, const T* src, size_t count) {
  int rc = dalloc(ctx, p, count);
  if (rc) return rc;
  if (count) HIPC(ctx, hipMemcpyAsync(*p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  return KSG_OK;
}

template <typename T>
int upc(ksg_ctx* ctx, const T*& field, const T* src, size_t count) {
  T* p = nullptr;
  int rc = upload(ctx, &p, src, count);
  field = p;
  return rc;
}

void free_all(ksg_ctx* ctx) {
  for (void* p : ctx->allocs) (void)hipFree(p);
  ctx->allocs.clear();
}

// Which kernel configuration to launch.
int launch_queue(ksg_ctx* ctx, QueueArgs& a, int n_replicas, int block) {
  (void)hipGetLastError();
  HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  if (block == 1024)
    hipLaunchKernelGGL(ksg_queue_kernel<1024>, dim3(n_replicas), dim3(1024), 0, ctx->stream, a);
  else if (block == 512)
    hipLaunchKernelGGL(ksg_queue_kernel<512>, dim3(n_replicas), dim3(512), 0, ctx->stream, a);
  else
    hipLaunchKernelGGL(ksg_queue_kernel<256>, dim3(n_replicas), dim3(256), 0, ctx->stream, a);
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  return KSG_OK;
}

int check_ready(ksg_ctx* ctx) {
  if (!ctx) return KSG_E_INVALID;
  if (!ctx->have_nodes || !ctx->have_wl || !ctx->have_prof)
    return fail(ctx, KSG_E_STATE, "profile, nodes and workload must be loaded first");
  if (ctx->max_blob > KSG_BLOB_MAX) return fail(ctx, KSG_E_UNSUPPORTED, "pod program blob exceeds LDS budget");
  return KSG_OK;
}

// PodTopologySpread / InterPodAffinity kernels are not in this build yet: refuse
// pods that need them instead of computing something else.
int check_supported(ksg_ctx* ctx, const ksg_profile& prof, int first, int count) {
  bool pts = false, ipa = false;
  for (int k = 0; k < prof.n_filter; k++) {
    pts |= prof.filter_order[k] == KSG_PL_POD_TOPOLOGY_SPREAD;
    ipa |= prof.filter_order[k] == KSG_PL_INTER_POD_AFFINITY;
  }
  pts |= (prof.score_mask >> KSG_PL_POD_TOPOLOGY_SPREAD) & 1u;
  ipa |= (prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u;
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if ((pts && p.pts >= 0) || (ipa && p.ipa >= 0))
      return fail(ctx, KSG_E_UNSUPPORTED, "PodTopologySpread/InterPodAffinity terms are not implemented in this build");
  }
  return KSG_OK;
}

QueueArgs base_args(ksg_ctx* ctx) {
  QueueArgs a{};
  a.c = ctx->c;
  a.st = ctx->st;
  a.pods = ctx->d_pods;
  a.prog = ctx->d_prog;
  return a;
}

}  // namespace

extern "C" {

int ksg_abi_version(void) { return KSG_ABI_VERSION; }

int ksg_open(int device, ksg_ctx** out) {
  if (!out) return KSG_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KSG_E_DEVICE;
  if (device < 0 || device >= ndev) return KSG_E_INVALID;
  ksg_ctx* ctx = new ksg_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return KSG_E_DEVICE;
  }
  *out = ctx;
  return KSG_OK;
}

int ksg_close(ksg_ctx* ctx) {
  if (!ctx) return KSG_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  free_all(ctx);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return KSG_OK;
}

const char* ksg_last_error(ksg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ksg_set_profile(ksg_ctx* ctx, const ksg_profile* prof) {
  if (!ctx || !prof) return KSG_E_INVALID;
  if (prof->n_filter < 0 || prof->n_filter > KSG_NPLUGINS || prof->fit_n < 0 || prof->fit_n > KSG_MAX_RES ||
      prof->ba_n < 0 || prof->ba_n > KSG_MAX_RES)
    return fail(ctx, KSG_E_INVALID, "profile field out of range");
  ctx->prof = *prof;
  ctx->have_prof = true;
  return KSG_OK;
}

int ksg_load_nodes(ksg_ctx* ctx, const ksg_nodes* nd, const ksg_topology* tp) {
  if (!ctx || !nd || !tp) return KSG_E_INVALID;
  HIPC(ctx, hipSetDevice(ctx->device));
  if (nd->n_nodes <= 0 || nd->n_res < 3 || nd->n_res > KSG_MAX_RES)
    return fail(ctx, KSG_E_INVALID, "bad node table sizes");
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  free_all(ctx);
  ctx->have_nodes = ctx->have_wl = false;
  const int N = nd->n_nodes, R = nd->n_res, L = std::max(nd->n_label_cols, 1);
  DevCluster& c = ctx->c;
  c = DevCluster{};
  c.N = N; c.R = R; c.L = nd->n_label_cols; c.T = nd->max_taints; c.I = nd->max_images;
  c.V = nd->n_taint_vocab; c.W = std::max(1, (nd->n_taint_vocab + 31) / 32);
  int rc = 0;
#define UP(field, src, cnt) if ((rc = upc(ctx, c.field, src, cnt))) return rc
  UP(alloc, nd->alloc, (size_t)R * N);
  UP(allowed, nd->allowed_pods, N);
  UP(unsched, nd->unschedulable, N);
  UP(label_val, nd->label_val, (size_t)L * N);
  UP(label_num, nd->label_num, (size_t)L * N);
  UP(label_num_ok, nd->label_num_ok, (size_t)L * N);
  UP(taints, nd->taints, (size_t)c.T * N);
  UP(taint_effect, nd->taint_effect, (size_t)std::max(c.V, 1));
  UP(images, nd->images, (size_t)c.I * N);
  c.S = tp->n_selectors;
  c.n_tmpl = tp->n_templates;
  const int nt = std::max(tp->n_templates, 1);
  UP(tmpl_col, tp->tmpl_col, nt);
  UP(tmpl_kind, tp->tmpl_kind, nt);
  UP(tmpl_weight, tp->tmpl_weight, nt);
  UP(col_vocab, tp->col_vocab, L);
  UP(col_unique, tp->col_unique, L);
  UP(log_table, tp->log_table, tp->log_n);
  c.log_n = tp->log_n;
  // template tables: one segment of col_vocab[col] words per template
  std::vector<int32_t> off(nt, 0);
  size_t total = 0;
  for (int t = 0; t < tp->n_templates; t++) {
    off[t] = (int32_t)total;
    total += (size_t)std::max(tp->col_vocab[tp->tmpl_col[t]], 1);
  }
  ctx->tab_words = std::max<size_t>(total, 1);
  UP(tmpl_off, off.data(), nt);
#undef UP
  // replica-0 state
  DevState& st = ctx->st;
  st = DevState{};
  if ((rc = upload(ctx, &st.requested, nd->requested, (size_t)R * N))) return rc;
  if ((rc = upload(ctx, &st.nonzero, nd->nonzero, (size_t)2 * N))) return rc;
  if ((rc = upload(ctx, &st.pod_count, nd->pod_count, N))) return rc;
  if ((rc = dalloc(ctx, &st.cnt, (size_t)std::max(c.S, 1) * N))) return rc;
  if ((rc = dalloc(ctx, &st.tab, ctx->tab_words))) return rc;
  if ((rc = dalloc(ctx, &st.tmpl_total, nt))) return rc;
  if ((rc = dalloc(ctx, &st.partial, N))) return rc;
  if ((rc = dalloc(ctx, &st.sraw, (size_t)4 * N))) return rc;
  HIPC(ctx, hipMemsetAsync(st.cnt, 0, sizeof(int32_t) * std::max(c.S, 1) * (size_t)N, ctx->stream));
  HIPC(ctx, hipMemsetAsync(st.tab, 0, sizeof(int32_t) * ctx->tab_words, ctx->stream));
  HIPC(ctx, hipMemsetAsync(st.tmpl_total, 0, sizeof(int32_t) * nt, ctx->stream));
  if ((rc = upload(ctx, &ctx->d_req0, nd->requested, (size_t)R * N))) return rc;
  if ((rc = upload(ctx, &ctx->d_nz0, nd->nonzero, (size_t)2 * N))) return rc;
  if ((rc = upload(ctx, &ctx->d_pc0, nd->pod_count, N))) return rc;
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  ctx->have_nodes = true;
  return KSG_OK;
}

int ksg_load_workload(ksg_ctx* ctx, const ksg_workload* wl) {
  if (!ctx || !wl || !wl->pods || wl->n_pods < 0 || wl->prog_len < 0) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "load nodes before the workload");
  HIPC(ctx, hipSetDevice(ctx->device));
  ctx->h_pods.assign(wl->pods, wl->pods + wl->n_pods);
  ctx->max_blob = 0;
  for (const ksg_pod& p : ctx->h_pods) {
    ctx->max_blob = std::max(ctx->max_blob, p.blob_len);
    if (p.blob < 0 || (int64_t)p.blob + p.blob_len > wl->prog_len)
      return fail(ctx, KSG_E_INVALID, "pod blob outside the program pool");
    if (p.node_set >= 0 && (int64_t)p.node_set + (ctx->c.N + 31) / 32 > wl->prog_len)
      return fail(ctx, KSG_E_INVALID, "node set outside the program pool");
  }
  int rc;
  if ((rc = upload(ctx, &ctx->d_pods, wl->pods, std::max(wl->n_pods, 1)))) return rc;
  if ((rc = upload(ctx, &ctx->d_prog, wl->prog, (size_t)std::max<int64_t>(wl->prog_len, 1)))) return rc;
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_pods = wl->n_pods;
  ctx->have_wl = true;
  return KSG_OK;
}

static int run_internal(ksg_ctx* ctx, int32_t first, int32_t count, int do_commit, int32_t* placements,
                        ksg_result* results, ksg_capture* cap) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (first < 0 || count < 0 || first + count > ctx->n_pods) return fail(ctx, KSG_E_INVALID, "pod range");
  if ((rc = check_supported(ctx, ctx->prof, first, count))) return rc;
  if (count == 0) return KSG_OK;
  HIPC(ctx, hipSetDevice(ctx->device));
  const size_t N = ctx->c.N;
  QueueArgs a = base_args(ctx);
  a.first = first;
  a.count = count;
  a.do_commit = do_commit;
  ksg_profile* d_prof = nullptr;
  int32_t* d_pl = nullptr;
  ksg_result* d_res = nullptr;
  std::vector<void*> tmp;
  auto cleanup = [&]() { for (void* p : tmp) (void)hipFree(p); };
  auto talloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 8));
    if (e == hipSuccess) tmp.push_back(*p);
    return e;
  };
#define TA(p, bytes) do { hipError_t _e = talloc((void**)(p), (bytes)); if (_e != hipSuccess) { cleanup(); return fail(ctx, KSG_E_NOMEM, hipGetErrorString(_e)); } } while (0)
  TA(&d_prof, sizeof(ksg_profile));
  TA(&d_pl, sizeof(int32_t) * count);
  if (results) TA(&d_res, sizeof(ksg_result) * count);
  a.profiles = d_prof;
  a.placements = d_pl;
  a.results = d_res;
  const bool want_cap = cap && (cap->fstatus || cap->raw || cap->norm || cap->total);
  if (want_cap) {
    TA(&a.cap_fstatus, sizeof(uint32_t) * N * count);
    TA(&a.cap_raw, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    TA(&a.cap_norm, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    TA(&a.cap_total, sizeof(int64_t) * N * count);
    (void)hipMemsetAsync(a.cap_raw, 0, sizeof(int64_t) * N * KSG_NPLUGINS * count, ctx->stream);
    (void)hipMemsetAsync(a.cap_norm, 0, sizeof(int64_t) * N * KSG_NPLUGINS * count, ctx->stream);
    (void)hipMemsetAsync(a.cap_total, 0, sizeof(int64_t) * N * count, ctx->stream);
  }
#undef TA
  hipError_t e = hipMemcpyAsync(d_prof, &ctx->prof, sizeof(ksg_profile), hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) { cleanup(); return fail(ctx, KSG_E_DEVICE, hipGetErrorString(e)); }
  const int block = N >= 2048 ? 1024 : (N >= 512 ? 512 : 256);
  rc = launch_queue(ctx, a, 1, block);
  if (rc) { cleanup(); return rc; }
  auto d2h = [&](void* dst, const void* src, size_t bytes) -> bool {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess;
  };
  bool ok = true;
  if (placements) ok &= d2h(placements, d_pl, sizeof(int32_t) * count);
  if (results) ok &= d2h(results, d_res, sizeof(ksg_result) * count);
  if (want_cap) {
    if (cap->fstatus) ok &= d2h(cap->fstatus, a.cap_fstatus, sizeof(uint32_t) * N * count);
    if (cap->raw) ok &= d2h(cap->raw, a.cap_raw, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    if (cap->norm) ok &= d2h(cap->norm, a.cap_norm, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    if (cap->total) ok &= d2h(cap->total, a.cap_total, sizeof(int64_t) * N * count);
  }
  e = hipStreamSynchronize(ctx->stream);
  float ms = 0;
  if (e == hipSuccess) (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_ms = ms;
  cleanup();
  if (e != hipSuccess || !ok) return fail(ctx, KSG_E_DEVICE, std::string("queue kernel: ") + hipGetErrorString(e));
  return KSG_OK;
}

int ksg_eval(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap) {
  if (!res) return fail(ctx, KSG_E_INVALID, "null result");
  int32_t pl;
  return run_internal(ctx, pod, 1, 0, &pl, res, cap);
}

int ksg_run_queue(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                  ksg_capture* cap) {
  return run_internal(ctx, first, count, 1, placements, results, cap);
}

int ksg_commit(ksg_ctx* ctx, int32_t pod, int32_t node) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods || node < 0 || node >= ctx->c.N) return fail(ctx, KSG_E_INVALID, "commit range");
  HIPC(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(ksg_commit_kernel, dim3(1), dim3(64), 0, ctx->stream, ctx->c, ctx->st, ctx->d_pods,
                     ctx->d_prog, pod, node);
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

int ksg_run_replicas(ksg_ctx* ctx, const ksg_profile* profiles, int32_t n_replicas, int32_t first, int32_t count,
                     int32_t* placements, ksg_replica_summary* summaries) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!profiles || n_replicas <= 0 || first < 0 || count < 0 || first + count > ctx->n_pods || !placements)
    return fail(ctx, KSG_E_INVALID, "replica arguments");
  for (int r = 0; r < n_replicas; r++)
    if ((rc = check_supported(ctx, profiles[r], first, count))) return rc;
  HIPC(ctx, hipSetDevice(ctx->device));
  const DevCluster& c = ctx->c;
  const size_t N = c.N, R = c.R, S = std::max(c.S, 1), NT = std::max(c.n_tmpl, 1);
  const size_t RR = n_replicas;
  QueueArgs a = base_args(ctx);
  a.first = first;
  a.count = count;
  a.do_commit = 1;
  std::vector<void*> tmp;
  auto cleanup = [&]() { for (void* p : tmp) (void)hipFree(p); };
  auto talloc = [&](void** p, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 8));
    if (e == hipSuccess) tmp.push_back(*p);
    return e;
  };
#define TA(p, bytes) do { hipError_t _e = talloc((void**)(p), (bytes)); if (_e != hipSuccess) { cleanup(); return fail(ctx, KSG_E_NOMEM, hipGetErrorString(_e)); } } while (0)
  DevState& s = a.st;
  s.stride_req = R * N; s.stride_nz = 2 * N; s.stride_pc = N; s.stride_cnt = S * N; s.stride_tab = ctx->tab_words;
  s.stride_tt = NT; s.stride_part = N; s.stride_sraw = 4 * N;
  TA(&s.requested, 8 * RR * s.stride_req);
  TA(&s.nonzero, 8 * RR * s.stride_nz);
  TA(&s.pod_count, 4 * RR * s.stride_pc);
  TA(&s.cnt, 4 * RR * s.stride_cnt);
  TA(&s.tab, 4 * RR * s.stride_tab);
  TA(&s.tmpl_total, 4 * RR * s.stride_tt);
  TA(&s.partial, 8 * RR * s.stride_part);
  TA(&s.sraw, 8 * RR * s.stride_sraw);
  ksg_profile* d_prof;
  int32_t* d_pl;
  TA(&d_prof, sizeof(ksg_profile) * RR);
  TA(&d_pl, sizeof(int32_t) * RR * count);
#undef TA
  bool ok = true;
  for (size_t r = 0; r < RR; r++) {  // every replica starts from the ctx's current state
    ok &= hipMemcpyAsync(s.requested + r * s.stride_req, ctx->st.requested, 8 * s.stride_req, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
    ok &= hipMemcpyAsync(s.nonzero + r * s.stride_nz, ctx->st.nonzero, 8 * s.stride_nz, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
    ok &= hipMemcpyAsync(s.pod_count + r * s.stride_pc, ctx->st.pod_count, 4 * s.stride_pc, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
    ok &= hipMemcpyAsync(s.cnt + r * s.stride_cnt, ctx->st.cnt, 4 * s.stride_cnt, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
    ok &= hipMemcpyAsync(s.tab + r * s.stride_tab, ctx->st.tab, 4 * s.stride_tab, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
    ok &= hipMemcpyAsync(s.tmpl_total + r * s.stride_tt, ctx->st.tmpl_total, 4 * s.stride_tt, hipMemcpyDeviceToDevice, ctx->stream) == hipSuccess;
  }
  ok &= hipMemcpyAsync(d_prof, profiles, sizeof(ksg_profile) * RR, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
  if (!ok) { cleanup(); return fail(ctx, KSG_E_DEVICE, "replica state copy"); }
  a.profiles = d_prof;
  a.placements = d_pl;
  a.results = nullptr;
  const int block = N >= 8192 ? 512 : 256;
  rc = launch_queue(ctx, a, (int)RR, block);
  if (rc) { cleanup(); return rc; }
  ok = hipMemcpyAsync(placements, d_pl, sizeof(int32_t) * RR * count, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess;
  std::vector<int64_t> req_cpu, req_mem;
  if (summaries) {
    req_cpu.resize(RR * s.stride_req);
    ok &= hipMemcpyAsync(req_cpu.data(), s.requested, 8 * RR * s.stride_req, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess;
  }
  hipError_t e = hipStreamSynchronize(ctx->stream);
  float ms = 0;
  if (e == hipSuccess) (void)hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  ctx->last_ms = ms;
  cleanup();
  if (e != hipSuccess || !ok) return fail(ctx, KSG_E_DEVICE, std::string("replica kernel: ") + hipGetErrorString(e));
  if (summaries) {
    for (size_t r = 0; r < RR; r++) {
      ksg_replica_summary& sm = summaries[r];
      sm = ksg_replica_summary{};
      uint64_t h = 1469598103934665603ull;
      for (int k = 0; k < count; k++) {
        int32_t v = placements[r * count + k];
        (v >= 0 ? sm.scheduled : sm.unschedulable) += 1;
        for (int b = 0; b < 4; b++) { h ^= (uint8_t)(((uint32_t)v) >> (8 * b)); h *= 1099511628211ull; }
      }
      sm.placement_hash = h;
      for (size_t n = 0; n < N; n++) {
        sm.cpu_requested += req_cpu[r * s.stride_req + n];
        sm.mem_requested += req_cpu[r * s.stride_req + N + n];
      }
    }
  }
  return KSG_OK;
}

int ksg_read_state(ksg_ctx* ctx, ksg_node_state* out) {
  if (!ctx || !out) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "no nodes loaded");
  HIPC(ctx, hipSetDevice(ctx->device));
  const size_t N = ctx->c.N, R = ctx->c.R;
  if (out->requested) HIPC(ctx, hipMemcpyAsync(out->requested, ctx->st.requested, 8 * R * N, hipMemcpyDeviceToHost, ctx->stream));
  if (out->nonzero) HIPC(ctx, hipMemcpyAsync(out->nonzero, ctx->st.nonzero, 16 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (out->pod_count) HIPC(ctx, hipMemcpyAsync(out->pod_count, ctx->st.pod_count, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

int ksg_reset_state(ksg_ctx* ctx) {
  if (!ctx) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "no nodes loaded");
  HIPC(ctx, hipSetDevice(ctx->device));
  const size_t N = ctx->c.N, R = ctx->c.R;
  HIPC(ctx, hipMemcpyAsync(ctx->st.requested, ctx->d_req0, 8 * R * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(ctx->st.nonzero, ctx->d_nz0, 16 * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(ctx->st.pod_count, ctx->d_pc0, 4 * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.cnt, 0, 4 * std::max(ctx->c.S, 1) * N, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.tab, 0, 4 * ctx->tab_words, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.tmpl_total, 0, 4 * std::max(ctx->c.n_tmpl, 1), ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

int ksg_last_kernel_ms(ksg_ctx* ctx, double* ms) {
  if (!ctx || !ms) return KSG_E_INVALID;
  *ms = ctx->last_ms;
  return KSG_OK;
}

}  // extern "C"
