// The per-cycle evaluation (ksg_eval's fast path, the Go shim's one call per
// scheduling cycle), included by ksched.hip inside its anonymous namespace.
//
// One launch, results written straight into pinned host memory, completion
// signalled by a flag the host polls: no copy launch, no event, no second
// kernel.  N / 256 workgroups:
//
//   every workgroup   its nodes' Filter status words and raw score rows (host
//                     memory), a packed record per node (device memory,
//                     agent-scope stores) and its partial feasible count /
//                     TaintToleration and NodeAffinity maxima / lowest
//                     feasible index (its own slot, agent-scope stores); then
//                     one arrival on a device counter
//   the last arrival  folds the slots, normalises TaintToleration and
//                     NodeAffinity over every node from the records, writes
//                     the normalised rows and totals, the selectHost argmax,
//                     the statistics slot, resets the counter and stores the
//                     call's sequence number into the host flag
//
// Hand-offs between workgroups follow ksched_sweep.h (gst / gld: agent-scope
// stores and loads, no cache maintenance); what the host reads is ordered by a
// system-scope fence in every workgroup before its arrival (its host stores)
// and in the last one before the flag.  Same arithmetic as ksg_capture_eval +
// ksg_capture_norm (nb = 1, nothing assumed), bit for bit.

struct CycPart {   // one workgroup's partial statistics
  int32_t nfeas, max_t, max_a, lo;   // lo = max over its feasible nodes of N - n
};

struct CycArgs {
  DevCluster c;
  DevState st;
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* prof;
  int32_t pod;
  int32_t n_rows, n_normrows;        // score rows (the normalising ones first)
  int32_t rows[KSG_NPLUGINS];
  int32_t narrow;                    // rows are int32 (host-checked) instead of int64
  // host outputs (fine-grained pinned memory, device addresses)
  uint32_t* h_fs;                    // [N]
  char* h_raw;                       // [n_rows][N]
  char* h_tot;                       // [N]
  char* h_norm;                      // [n_normrows][N]
  int32_t* h_stats;                  // [4] nfeas, max taint, max node affinity, max (N - n)
  unsigned long long* h_best;        // selectHost key
  uint32_t* h_err;                   // a normalised score left [0, 100]
  unsigned* h_flag;                  // = seq once everything above is written
  unsigned seq;
  // device scratch
  uint64_t* rec;                     // [N]
  CycPart* parts;                    // [G]
  unsigned* done;                    // arrivals of this call (reset to 0 by the last one)
  // a staged append of this pod (ksg_capture_eval's spod fields)
  const ksg_pod* spod;
  const int32_t* sprog;
  int64_t sbase, slen;
  ksg_pod* wpods;
  int32_t* wprog;
};

__device__ __forceinline__ void cyc_put(char* base, size_t idx, int64_t v, bool narrow) {
  if (narrow) reinterpret_cast<int32_t*>(base)[idx] = (int32_t)v;
  else reinterpret_cast<int64_t*>(base)[idx] = v;
}

__global__ __launch_bounds__(256) void ksg_eval_cycle(CycArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ int32_t s_st[4][4];
  __shared__ unsigned long long s_key[4];
  __shared__ uint32_t s_err[4];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N;
  const size_t NN = N;
  const bool narrow = a.narrow != 0;
  if (tid < (int)(sizeof(ksg_profile) / 4))
    reinterpret_cast<int32_t*>(&s_prof)[tid] = reinterpret_cast<const int32_t*>(a.prof)[tid];
  const int32_t* gprog = a.prog;
  if (a.spod) {   // the staged append: read it from the host buffer; workgroup 0 copies it to the device
    if (tid < (int)(sizeof(ksg_pod) / 4))
      reinterpret_cast<int32_t*>(&s_pod)[tid] = reinterpret_cast<const int32_t*>(a.spod)[tid];
    __syncthreads();
    const int64_t boff = s_pod.blob - a.sbase;
    for (int i = tid; i < s_pod.blob_len; i += 256) s_blob[i] = a.sprog[boff + i];
    gprog = a.sprog - a.sbase;
    if (blockIdx.x == 0) {
      if (tid < (int)(sizeof(ksg_pod) / 4))
        reinterpret_cast<int32_t*>(a.wpods)[tid] = reinterpret_cast<const int32_t*>(&s_pod)[tid];
      for (int64_t i = tid; i < a.slen; i += 256) a.wprog[i] = a.sprog[i];
    }
  } else {
    stage_pod<256>(a.pods, a.prog, a.pod, &s_pod, s_blob);
  }
  __syncthreads();
  const PodView v = make_view(c, s_prof, s_pod, s_blob, gprog, false, a.st.ports);

  // ---- every workgroup: its nodes ------------------------------------------------
  const int n = blockIdx.x * 256 + tid;
  int32_t feas = 0, mt = 0, ma = 0, lo = 0;
  if (n < N) {
    NodeCols L;
    load_cols(c, a.st.requested, a.st.nonzero, a.st.pod_count, n, L);
    int64_t lraw[KSG_NPLUGINS] = {};
    const NodeEval e = eval_node_src(c, s_prof, v, GNode{&c, n}, L, n, nullptr, nullptr, nullptr, lraw);
    a.h_fs[n] = e.st;
    gst(&a.rec[n], pack_rec(e));
    const bool ok = e.st == 0;
    for (int q = 0; q < a.n_rows; q++) {
      const int pl = a.rows[q];
      int64_t x = 0;
      switch (pl) {   // the node-local plugins; the others are not on this path
        case KSG_PL_NODE_RESOURCES_FIT: x = lraw[KSG_PL_NODE_RESOURCES_FIT]; break;
        case KSG_PL_BALANCED_ALLOCATION: x = lraw[KSG_PL_BALANCED_ALLOCATION]; break;
        case KSG_PL_IMAGE_LOCALITY: x = lraw[KSG_PL_IMAGE_LOCALITY]; break;
        case KSG_PL_TAINT_TOLERATION: x = lraw[KSG_PL_TAINT_TOLERATION]; break;
        case KSG_PL_NODE_AFFINITY: x = lraw[KSG_PL_NODE_AFFINITY]; break;
        default: break;
      }
      x = ok && ((v.smask >> pl) & 1u) ? x : 0;
      cyc_put(a.h_raw, (size_t)q * NN + n, x, narrow);   // a pod with < 2 feasible nodes: zeroed below
    }
    if (ok) {
      feas = 1;
      mt = (int32_t)e.rt;
      ma = (int32_t)e.ra;
      lo = N - n;
    }
  }
  feas = wave_sum32(feas);
  mt = (int32_t)wave_max64(mt);
  ma = (int32_t)wave_max64(ma);
  lo = (int32_t)wave_max64(lo);
  if (lane == 0) { s_st[0][wv] = feas; s_st[1][wv] = mt; s_st[2][wv] = ma; s_st[3][wv] = lo; }
  __syncthreads();
  if (tid == 0) {
    int32_t f = 0, t = 0, m = 0, l = 0;
    for (int i = 0; i < 4; i++) {
      f += s_st[0][i];
      t = max(t, s_st[1][i]);
      m = max(m, s_st[2][i]);
      l = max(l, s_st[3][i]);
    }
    CycPart* pp = a.parts + blockIdx.x;
    gst(&pp->nfeas, f);
    gst(&pp->max_t, t);
    gst(&pp->max_a, m);
    gst(&pp->lo, l);
  }
  // every wave's host and hand-off stores performed before the arrival
  __threadfence_system();
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)a.done, 1u,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;

  // ---- the last arrival: fold, normalise, select ------------------------------------
  int32_t f = 0, t = 0, m = 0, l = 0;
  for (int b = tid; b < (int)gridDim.x; b += 256) {
    const CycPart* pp = a.parts + b;
    f += gld(&pp->nfeas);
    t = max(t, gld(&pp->max_t));
    m = max(m, gld(&pp->max_a));
    l = max(l, gld(&pp->lo));
  }
  f = wave_sum32(f);
  t = (int32_t)wave_max64(t);
  m = (int32_t)wave_max64(m);
  l = (int32_t)wave_max64(l);
  __syncthreads();   // s_st reuse
  if (lane == 0) { s_st[0][wv] = f; s_st[1][wv] = t; s_st[2][wv] = m; s_st[3][wv] = l; }
  __syncthreads();
  int32_t nfeas = 0, max_t = 0, max_a = 0, low = 0;
  for (int i = 0; i < 4; i++) {
    nfeas += s_st[0][i];
    max_t = max(max_t, s_st[1][i]);
    max_a = max(max_a, s_st[2][i]);
    low = max(low, s_st[3][i]);
  }
  uint64_t key = 0;
  uint32_t err = 0;
  for (int k = tid; k < N; k += 256) {
    const uint64_t x = gld(&a.rec[k]);
    int64_t total = 0, nt = 0, na = 0;
    if (nfeas >= 2 && (x >> 63)) {
      total = total_score(v, (uint32_t)x, (x >> 48) & 0xff, (x >> 32) & 0xffff, max_t, max_a, err, &nt, &na);
      const uint64_t kk = argmax_key(total, k);
      key = kk > key ? kk : key;
    }
    cyc_put(a.h_tot, k, total, narrow);
    for (int q = 0; q < a.n_rows; q++) {
      const int pl = a.rows[q];
      if (nfeas < 2) {   // fewer than two feasible nodes: no Score runs, nothing recorded
        cyc_put(a.h_raw, (size_t)q * NN + k, 0, narrow);
        if (q < a.n_normrows) cyc_put(a.h_norm, (size_t)q * NN + k, 0, narrow);
      } else if (q < a.n_normrows) {
        cyc_put(a.h_norm, (size_t)q * NN + k, pl == KSG_PL_TAINT_TOLERATION ? nt : na, narrow);
      }
    }
  }
  key = wave_max_u64(key);
  err = wave_or32(err);
  if (lane == 0) { s_key[wv] = key; s_err[wv] = err; }
  __syncthreads();
  if (tid == 0) {
    uint64_t k = 0;
    uint32_t e = 0;
    for (int i = 0; i < 4; i++) { k = s_key[i] > k ? s_key[i] : k; e |= s_err[i]; }
    a.h_stats[0] = nfeas;
    a.h_stats[1] = max_t;
    a.h_stats[2] = max_a;
    a.h_stats[3] = low;
    *a.h_best = k;
    *a.h_err = e;
    gst(a.done, 0u);   // the next call's arrivals
  }
  __threadfence_system();
  __syncthreads();
  if (tid == 0) __hip_atomic_store(a.h_flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
