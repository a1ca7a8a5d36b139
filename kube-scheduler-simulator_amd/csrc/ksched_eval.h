// The per-cycle evaluation kernel (included by ksched.hip inside its anonymous
// namespace, after ksched_sweep.h, whose agent-scope helpers it uses).

// The per-cycle evaluation in ONE launch (ksg_eval's chip-wide path): the
// body of ksg_capture_eval, a grid barrier, the body of ksg_capture_norm.
// Workgroup x owns nodes x * 256 + tid in both halves, so a node's packed
// record stays in its lane's registers; only the pod's statistics cross
// workgroups, through agent-scope atomics read back with agent-scope loads
// after the barrier (the fence-free hand-off of ksched_sweep.h,
// arrive_and_wait_sc1).  Launched cooperatively (co-residency of the N / 256
// workgroups guaranteed); bar is a monotonic arrival counter (the caller
// passes the count this call completes at), the poll is bounded.
__device__ __forceinline__ void agent_max(int32_t* p, int32_t v) {
  __hip_atomic_fetch_max((__attribute__((address_space(1))) int32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void ksg_eval_fused(CapArgs a, unsigned* bar, unsigned* timeout, unsigned target0) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ int32_t s_st[4][4];
  __shared__ unsigned long long s_key[4];
  __shared__ uint32_t s_err[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N;
  const size_t NN = N;
  if (tid < (int)(sizeof(ksg_profile) / 4))
    reinterpret_cast<int32_t*>(&s_prof)[tid] = reinterpret_cast<const int32_t*>(a.prof)[tid];
  if (a.next && blockIdx.x == 0 && tid < 8) a.next[tid] = 0;   // the next call's slot
  stage_pod<256>(a.pods, a.prog, a.b0, &s_pod, s_blob);
  __syncthreads();
  const PodView v = make_view(c, s_prof, s_pod, s_blob, a.prog, false, a.st.ports);
  const int n = blockIdx.x * 256 + tid;
  // ---- the ksg_capture_eval half: filters, node-local raw scores ------------
  uint64_t x = 0;
  int32_t feas = 0, mt = 0, ma = 0, lo = 0;
  if (n < N) {
    NodeCols L;
    load_cols(c, a.st.requested, a.st.nonzero, a.st.pod_count, n, L);
    int64_t lraw[KSG_NPLUGINS] = {};
    const NodeEval e = eval_node_src(c, s_prof, v, GNode{&c, n}, L, n, nullptr, nullptr, nullptr, lraw);
    a.fstatus[n] = e.st;
    x = pack_rec(e);
    const bool ok = e.st == 0;
    for (int q = 0; q < a.n_rows; q++) {
      const int pl = a.rows[q];
      int64_t r = 0;
      switch (pl) {
        case KSG_PL_NODE_RESOURCES_FIT: r = lraw[KSG_PL_NODE_RESOURCES_FIT]; break;
        case KSG_PL_BALANCED_ALLOCATION: r = lraw[KSG_PL_BALANCED_ALLOCATION]; break;
        case KSG_PL_IMAGE_LOCALITY: r = lraw[KSG_PL_IMAGE_LOCALITY]; break;
        case KSG_PL_TAINT_TOLERATION: r = lraw[KSG_PL_TAINT_TOLERATION]; break;
        case KSG_PL_NODE_AFFINITY: r = lraw[KSG_PL_NODE_AFFINITY]; break;
        default: break;
      }
      r = ok && ((v.smask >> pl) & 1u) ? r : 0;
      cap_put(a.raw, (size_t)q * NN + n, r, a.narrow);
      if (pl != KSG_PL_TAINT_TOLERATION && pl != KSG_PL_NODE_AFFINITY) cap_put(a.norm, (size_t)q * NN + n, r, a.narrow);
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
    if (f) gadd(&a.stats[0], f);
    if (t) agent_max(&a.stats[1], t);
    if (m) agent_max(&a.stats[2], m);
    if (l) agent_max(&a.stats[3], l);
  }
  unsigned target = target0 - gridDim.x;
  if (!arrive_and_wait_sc1(bar, timeout, (int)gridDim.x, target)) return;
  // ---- the ksg_capture_norm half: normalise, weight, selectHost --------------
  const int32_t nfeas = gld(&a.stats[0]), max_t = gld(&a.stats[1]), max_a = gld(&a.stats[2]);
  uint64_t key = 0;
  uint32_t err = 0;
  int64_t total = 0, nt = 0, na = 0;
  if (n < N && nfeas >= 2 && (x >> 63)) {
    total = total_score(v, (uint32_t)x, (x >> 48) & 0xff, (x >> 32) & 0xffff, max_t, max_a, err, &nt, &na);
    key = argmax_key(total, n);
  }
  key = wave_max_u64(key);
  err = wave_or32(err);
  if (lane == 0) { s_key[wv] = key; s_err[wv] = err; }
  __syncthreads();
  if (tid == 0) {
    uint64_t k = 0;
    uint32_t e = 0;
    for (int i = 0; i < 4; i++) { k = s_key[i] > k ? s_key[i] : k; e |= s_err[i]; }
    if (k) __hip_atomic_fetch_max((__attribute__((address_space(1))) unsigned long long*)a.best, (unsigned long long)k,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e) __hip_atomic_fetch_or((__attribute__((address_space(1))) uint32_t*)a.err, e, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
  }
  if (n >= N) return;
  if (a.total) cap_put(a.total, n, total, a.narrow);
  for (int q = 0; q < a.n_rows; q++) {
    const int pl = a.rows[q];
    if (nfeas < 2) {   // fewer than two feasible nodes: no Score runs, nothing recorded
      cap_put(a.raw, (size_t)q * NN + n, 0, a.narrow);
      cap_put(a.norm, (size_t)q * NN + n, 0, a.narrow);
    } else if (pl == KSG_PL_TAINT_TOLERATION) {
      cap_put(a.norm, (size_t)q * NN + n, nt, a.narrow);
    } else if (pl == KSG_PL_NODE_AFFINITY) {
      cap_put(a.norm, (size_t)q * NN + n, na, a.narrow);
    }
  }
}
