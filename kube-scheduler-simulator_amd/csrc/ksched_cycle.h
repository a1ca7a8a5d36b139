// The per-cycle evaluation (ksg_eval's fast path, the Go shim's one call per
// scheduling cycle, wrappedplugin.go:388-548), included by ksched.hip inside
// its anonymous namespace.
//
// One launch of G = ceil(N / BLOCK) co-resident workgroups (cooperative
// launch), one node per lane, results written straight into the pinned,
// fine-grained host block the caller reads in place (ksg_eval_view):
//
//   phase 1 (every workgroup)  stage the pod into LDS; evaluate its nodes
//                              (filters in profile order, raw scores); store
//                              each node's status word and raw score rows to
//                              the host block at once (coalesced, in flight
//                              during the exchange); keep the packed record in
//                              registers; publish the workgroup's feasible
//                              count, TaintToleration / NodeAffinity maxima and
//                              lowest feasible index in its own slot
//   exchange                   grid barrier on per-workgroup flags (one
//                              128-byte line each, tagged with the call's
//                              sequence number, so nothing is reset per call)
//   phase 2 (every workgroup)  fold the G slots (every workgroup computes the
//                              same pod-wide values), normalise its own nodes
//                              (DefaultNormalizeScore), store the normalised
//                              rows and weighted totals, its selectHost key;
//                              a pod with < 2 feasible nodes ran no Score, so
//                              its raw rows are zeroed instead
//   completion                 every workgroup writes its selectHost key and
//                              error bits into its own record of the host
//                              block, then (after its rows) its done word =
//                              the call's sequence number; the host folds the
//                              G keys (no arrival counter, no last workgroup)
//
// No workgroup walks all N nodes and every row is written once.  The
// exchange follows ksched_sweep.h (gst / gld: agent-scope stores and loads,
// every wave drained before the workgroup barrier in front of the flag); the
// host-visible bytes are system-scope stores drained (vmcnt(0)) before the
// workgroup's done word.  Rows are 2, 4 or 8 bytes per value (the narrowest
// exact width, chosen by the host).  Same arithmetic as ksg_capture_eval +
// ksg_capture_norm (nb = 1, nothing assumed), bit for bit.

struct CycPart {   // one workgroup's phase-1 statistics
  int32_t nfeas, max_t, max_a, lo;   // lo = max over its feasible nodes of N - n
};
struct CycWg {     // one workgroup's record in the host block
  unsigned long long key;   // its selectHost key (0: no feasible node)
  uint32_t err;             // bit 0: a normalised score left [0, 100]; bit 1: the exchange timed out
  uint32_t done;            // = seq once every row of the workgroup and the two words above are written
};

// The launch arguments.  The prologue's fields come first and together: the
// kernel-argument segment is read with scalar loads, and fields the compiler
// reaches through separate branches cost one round trip each.
struct CycArgs {
  // ---- prologue ----
  const int32_t* psrc;               // the pod record: device pool or staged append
  const int32_t* bsrc;               // its program blob
  const int32_t* gprog;              // the program pool as the kernel sees it (node_set)
  const ksg_profile* prof;
  int32_t blob, blob_len;            // the pod's program blob (host copy of pods[pod].blob / blob_len)
  int32_t cm_node;                   // a deferred assume (ksg_commit of a pod without selectors, templates or
                                     // host ports) onto node cm_node, -1 none: its owner lane adds it first
  int64_t cm_req[KSG_MAX_RES];
  int64_t cm_nz_cpu, cm_nz_mem;
  // a staged append of this pod: workgroup 0 writes it to the device pool
  ksg_pod* wpods;                    // null: nothing staged
  int32_t* wprog;
  const int32_t* sprog;              // the staged words
  int64_t slen;
  // ---- evaluation ----
  DevCluster c;
  DevState st;
  int32_t n_rows, n_normrows;        // score rows (the normalising ones first)
  int32_t rows[KSG_NPLUGINS];
  int32_t es;                        // bytes per row value: 2, 4 or 8 (host range-checked)
  // host outputs (fine-grained pinned memory, device addresses)
  uint32_t* h_fs;                    // [N]
  char* h_raw;                       // [n_rows][N]
  char* h_tot;                       // [N]
  char* h_norm;                      // [n_normrows][N]
  int32_t* h_stats;                  // [4] nfeas, max taint, max node affinity, max (N - n) (workgroup 0)
  CycWg* h_wg;                       // [G]
  unsigned seq;
  // device scratch
  CycPart* parts;                    // [G]
  unsigned* flags;                   // [G][32]: workgroup g's exchange flag at [g * 32]
  unsigned* timeout;                 // sticky: an exchange poll gave up (reported to the host)
  unsigned long long* stamps;        // KSG_STAMPS builds: per-segment cycle sums of workgroup 0
};

#ifdef KSG_STAMPS
#define KSG_YSTAMP(seg)                                                       \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();               \
    if (tid == 0 && blockIdx.x == 0) { y_acc[seg] += _t - y_last; y_last = _t; } \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#else
#define KSG_YSTAMP(seg) do {} while (0)
#endif
// Grid exchange: workgroup g stores `seq` into its own flag line, wave 0 polls
// every flag until all hold `seq` (bounded; a timeout is sticky and reported).
template <int BLOCK>
__device__ __forceinline__ bool cyc_exchange(const CycArgs& a, int G) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its agent-scope stores are done
  __syncthreads();
  __shared__ int s_to;
  const int tid = threadIdx.x;
  if (tid < 64) {
    if (tid == 0) gst(&a.flags[(size_t)blockIdx.x * 32], a.seq);
    unsigned spins = 0;
    int to = 0;
    for (;;) {
      bool ok = true;
      for (int l = tid; l < G; l += 64) ok = ok && gld(&a.flags[(size_t)l * 32]) == a.seq;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22) || gld(a.timeout)) {
        if (tid == 0) gst(a.timeout, 1u);
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

template <int BLOCK, bool SYS>
__global__ __launch_bounds__(BLOCK) void ksg_eval_cycle(CycArgs a) {
  constexpr int NW = BLOCK / 64;
  constexpr int PW = (int)(sizeof(ksg_pod) / 4);
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ int32_t s_st[4][NW];
  __shared__ unsigned long long s_key[NW];
  __shared__ uint32_t s_err[NW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = (int)gridDim.x;
  const DevCluster& c = a.c;
  const int N = c.N;
  const size_t NN = N;
  const int es = a.es;
#ifdef KSG_STAMPS
  unsigned long long y_acc[10] = {}, y_last = __builtin_amdgcn_s_memtime();
#endif
  // Every load of the prologue is issued before the first wait: the pod
  // record and its program blob (offset and length come with the launch, so
  // the blob loads do not wait for the record) and this lane's node columns,
  // so the chain costs one memory latency.  The sources are host-resolved
  // pointers (no branch on the arguments: their scalar loads go out together).
  // The profile is read through the constant address space: every plugin
  // loop over it is a wave-uniform scalar load, not an LDS round trip per step.
  const ksg_profile& prof = *(const ksg_profile*)(const __attribute__((address_space(4))) ksg_profile*)a.prof;
  const int32_t* prec = a.psrc;
  const int32_t* bsrc = a.bsrc;
  const int32_t pw = tid < PW ? prec[tid] : 0;
  constexpr int BI = (KSG_BLOB_MAX + BLOCK - 1) / BLOCK;
  int32_t bw[BI];
#pragma unroll
  for (int u = 0; u < BI; u++) {
    const int i = tid + u * BLOCK;
    bw[u] = i < a.blob_len ? bsrc[i] : 0;
  }
  const int n = blockIdx.x * BLOCK + tid;
  const bool own = n < N;
  NodeCols L;
  if (own) load_cols(c, a.st.requested, a.st.nonzero, a.st.pod_count, n, L);
  if (tid < PW) reinterpret_cast<int32_t*>(&s_pod)[tid] = pw;
#pragma unroll
  for (int u = 0; u < BI; u++) {
    const int i = tid + u * BLOCK;
    if (i < a.blob_len) s_blob[i] = bw[u];
  }
  if (a.wpods && blockIdx.x == 0) {   // the staged append: workgroup 0 copies it to the device
    if (tid < PW) reinterpret_cast<int32_t*>(a.wpods)[tid] = pw;
    for (int64_t i = tid; i < a.slen; i += BLOCK) a.wprog[i] = a.sprog[i];
  }
  lds_barrier();   // LDS only: the node-column loads stay in flight
  // (after the barrier: only the owner lane's wave waits for its columns, where
  // its evaluation would wait for them anyway)
  if (own && n == a.cm_node) {   // the deferred assume: NodeInfo.AddPod on the lane's own node
#pragma unroll
    for (int r = 0; r < KSG_MAX_RES; r++)
      if (r < c.R) {
        L.req[r] += a.cm_req[r];
        a.st.requested[(size_t)r * NN + n] = L.req[r];
      }
    L.nz_cpu += a.cm_nz_cpu;
    L.nz_mem += a.cm_nz_mem;
    L.pod_count += 1;
    a.st.nonzero[n] = L.nz_cpu;
    a.st.nonzero[NN + n] = L.nz_mem;
    a.st.pod_count[n] = L.pod_count;
  }
  KSG_YSTAMP(0);
  const PodView v = make_view(c, prof, s_pod, s_blob, a.gprog, false, a.st.ports);

  // ---- phase 1: this workgroup's nodes ------------------------------------------------
  NodeEval e{KSG_FS_NOT_EVALUATED, 0, 0, 0, 0};
  int64_t lraw[KSG_NPLUGINS] = {};
  const CmProf cm = cm_prof(prof);
  if (own) e = eval_node_src(c, prof, v, GNode{&c, n}, L, n, nullptr, nullptr, nullptr, lraw, &cm);
  KSG_YSTAMP(1);
  const bool ok = own && e.st == 0;
  // the row value of score row q (node-local plugins only on this path)
  auto raw_of = [&](int q) -> int64_t {
    const int pl = a.rows[q];
    int64_t x = 0;
    switch (pl) {
      case KSG_PL_NODE_RESOURCES_FIT: x = lraw[KSG_PL_NODE_RESOURCES_FIT]; break;
      case KSG_PL_BALANCED_ALLOCATION: x = lraw[KSG_PL_BALANCED_ALLOCATION]; break;
      case KSG_PL_IMAGE_LOCALITY: x = lraw[KSG_PL_IMAGE_LOCALITY]; break;
      case KSG_PL_TAINT_TOLERATION: x = lraw[KSG_PL_TAINT_TOLERATION]; break;
      case KSG_PL_NODE_AFFINITY: x = lraw[KSG_PL_NODE_AFFINITY]; break;
      default: break;
    }
    return ok && ((v.smask >> pl) & 1u) ? x : 0;
  };
  int32_t feas = ok ? 1 : 0, mt = ok ? (int32_t)e.rt : 0, ma = ok ? (int32_t)e.ra : 0, lo = ok ? N - n : 0;
  feas = wave_sum32(feas);
  mt = (int32_t)wave_max64(mt);
  ma = (int32_t)wave_max64(ma);
  lo = (int32_t)wave_max64(lo);
  if (NW > 1) {
    if (lane == 0) { s_st[0][wv] = feas; s_st[1][wv] = mt; s_st[2][wv] = ma; s_st[3][wv] = lo; }
    __syncthreads();
    if (tid == 0)
      for (int i = 1; i < NW; i++) {
        feas += s_st[0][i];
        mt = max(mt, s_st[1][i]);
        ma = max(ma, s_st[2][i]);
        lo = max(lo, s_st[3][i]);
      }
  }
  if (tid == 0) {
    CycPart* pp = a.parts + blockIdx.x;
    gst(&pp->nfeas, feas);
    gst(&pp->max_t, mt);
    gst(&pp->max_a, ma);
    gst(&pp->lo, lo);
  }

  KSG_YSTAMP(2);
  // ---- exchange -------------------------------------------------------------------------
  const bool xok = cyc_exchange<BLOCK>(a, G);
  KSG_YSTAMP(3);

  // ---- phase 2: fold the slots, normalise this workgroup's nodes ------------------------
  int32_t nfeas = 0, max_t = 0, max_a = 0, low = 0;
  for (int b = tid; b < G; b += BLOCK) {
    const CycPart* pp = a.parts + b;
    nfeas += gld(&pp->nfeas);
    max_t = max(max_t, gld(&pp->max_t));
    max_a = max(max_a, gld(&pp->max_a));
    low = max(low, gld(&pp->lo));
  }
  nfeas = wave_sum32(nfeas);
  max_t = (int32_t)wave_max64(max_t);
  max_a = (int32_t)wave_max64(max_a);
  low = (int32_t)wave_max64(low);
  if (NW > 1) {
    __syncthreads();   // s_st reuse
    if (lane == 0) { s_st[0][wv] = nfeas; s_st[1][wv] = max_t; s_st[2][wv] = max_a; s_st[3][wv] = low; }
    __syncthreads();
    nfeas = 0; max_t = 0; max_a = 0; low = 0;
    for (int i = 0; i < NW; i++) {
      nfeas += s_st[0][i];
      max_t = max(max_t, s_st[1][i]);
      max_a = max(max_a, s_st[2][i]);
      low = max(low, s_st[3][i]);
    }
  }
  KSG_YSTAMP(4);
  // every row of this workgroup's nodes, written once (the exchange above
  // waited for nothing on the host link)
  uint64_t key = 0;
  uint32_t err = 0;
  if (own) {
    const bool scored = nfeas >= 2;   // fewer than two feasible nodes: no Score ran, nothing recorded
    int64_t total = 0, nt = 0, na = 0;
    if (scored && ok) {
      total = total_score(v, e.part, e.rt, e.ra, max_t, max_a, err, &nt, &na);
      key = argmax_key(total, n);
    }
    hst<SYS>(a.h_fs + n, e.st);
    for (int q = 0; q < a.n_rows; q++) cyc_put_es<SYS>(a.h_raw, (size_t)q * NN + n, scored ? raw_of(q) : 0, es);
    for (int q = 0; q < a.n_normrows; q++)
      cyc_put_es<SYS>(a.h_norm, (size_t)q * NN + n, a.rows[q] == KSG_PL_TAINT_TOLERATION ? nt : na, es);
    cyc_put_es<SYS>(a.h_tot, n, total, es);
  }
  key = wave_max_u64(key);
  err = wave_or32(err);
  if (NW > 1) {
    if (lane == 0) { s_key[wv] = key; s_err[wv] = err; }
    __syncthreads();
    if (tid == 0)
      for (int i = 1; i < NW; i++) { key = s_key[i] > key ? s_key[i] : key; err |= s_err[i]; }
  }
  host_release<SYS>();   // this wave's rows are written
  KSG_YSTAMP(5);
  __syncthreads();       // ... and every other wave's
  if (tid == 0) {
    CycWg* w = a.h_wg + blockIdx.x;
    hst<SYS>(&w->key, (unsigned long long)key);
    hst<SYS>(&w->err, err | (xok ? 0u : 2u));
    if (blockIdx.x == 0) {   // the pod-wide statistics (every workgroup folded the same values)
      hst<SYS>(a.h_stats + 0, nfeas);
      hst<SYS>(a.h_stats + 1, max_t);
      hst<SYS>(a.h_stats + 2, max_a);
      hst<SYS>(a.h_stats + 3, low);
    }
    host_release<SYS>();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&w->done, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  KSG_YSTAMP(6);
#ifdef KSG_STAMPS
  if (tid == 0 && blockIdx.x == 0 && a.stamps)
    for (int i = 0; i < 7; i++) atomicAdd(&a.stamps[i], y_acc[i]);
#endif
}
