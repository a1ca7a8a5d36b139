// Capture on the batched placement path (included by ksched.hip inside its
// anonymous namespace).
//
// The wrapped plugins record, per pod, every node's filter verdict and every
// score plugin's Score() / NormalizeScore() value (store.go:423-507).  The
// batched path decides placements without ever materialising those values,
// so a captured batch runs two extra kernels after its phase 2, when the
// state already holds the whole batch:
//
//   ksg_capture_eval  grid (node tiles, batch pods): pod j sees node n as the
//                     post-batch state minus the pods k >= j of the batch that
//                     were placed on n (exactly the state at pod j's turn);
//                     filter status word, node-local raw scores, packed record
//                     into the phase-1 record buffer (free after phase 2) and
//                     the pod's feasible count / TaintToleration and
//                     NodeAffinity maxima;
//   ksg_capture_norm  same grid: DefaultNormalizeScore of TaintToleration and
//                     NodeAffinity and the weighted total, for pods with >= 2
//                     feasible nodes (the others record no scores: their rows
//                     are zeroed, schedule_one.go skips Score with one node).
//
// Rows: only the profile's score plugins are written, in a compact
// [pod][row][node] layout (rows[q] = plugin id); the host copies each row into
// the caller's [pod][plugin][node] arrays.  Every written row gets every node
// (0 where the node is infeasible or the pod skipped the plugin), so no memset
// of the capture buffers is needed.

struct CapArgs {
  DevCluster c;
  DevState st;
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* prof;
  int32_t b0, nb, out0;          // batch = pods [b0, b0 + nb), output index of pod b0
  const int32_t* placements;     // [count] (this run)
  uint64_t* rec;                 // [nb][N] scratch (the phase-1 record buffer)
  int32_t* stats;                // [nb][4] nfeas, max taint, max node affinity, 0 (zeroed before the batch)
  int32_t n_rows;
  int32_t rows[KSG_NPLUGINS];    // plugin id of compact row q
  uint32_t* fstatus;             // [count][N]
  int64_t* raw;                  // [count][n_rows][N]
  int64_t* norm;                 // [count][n_rows][N]
  int64_t* total;                // [count][N]
  // per-cycle evaluation (ksg_eval's fast path, nb = 1, nothing assumed):
  // stats[3] = max over feasible nodes of N - n (lowest feasible index),
  // *best = selectHost's packed argmax key, *err = a normalised score left
  // [0, 100]; *next is the other call parity's slot, zeroed by block 0 of
  // ksg_capture_norm for the next call (no memset launch).  Null otherwise.
  unsigned long long* best;
  uint32_t* err;
  int32_t* next;                 // 8 words: the next call's stats[4], best, err
  int32_t narrow;                // raw / norm / total rows are int32 (the per-cycle path's copy-back; the
                                 // host checked every value fits) instead of int64
  // per-cycle evaluation of a pod whose append is still staged (ksched.hip
  // flush_stage): its record and program words [sbase, sbase + slen) are read
  // from the fine-grained host staging buffer, and workgroup (0, 0) writes them
  // to the device arrays (wpods = &pods[b0], wprog = &prog[sbase]) for the
  // kernels after this one.  Null otherwise.
  const ksg_pod* spod;
  const int32_t* sprog;
  int64_t sbase, slen;
  ksg_pod* wpods;
  int32_t* wprog;
};

// Row element idx of a capture array: int64, or int32 in the narrow form.
__device__ __forceinline__ void cap_put(int64_t* base, size_t idx, int64_t v, bool narrow) {
  if (narrow) reinterpret_cast<int32_t*>(base)[idx] = (int32_t)v;
  else base[idx] = v;
}

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_capture_eval(CapArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ int32_t s_pl[KSG_BATCH_MAX];
  __shared__ int32_t s_st[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = blockIdx.y;
  const DevCluster& c = a.c;
  const int N = c.N;
  const size_t NN = N;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.prof)[i_];
  for (int k = tid; k < a.nb; k += 256) s_pl[k] = a.placements[a.out0 + k];
  const int32_t* gprog = a.prog;
  if (a.spod) {   // the staged append (nb = 1)
    if (tid < (int)(sizeof(ksg_pod) / 4))
      reinterpret_cast<int32_t*>(&s_pod)[tid] = reinterpret_cast<const int32_t*>(a.spod)[tid];
    __syncthreads();
    const int64_t boff = s_pod.blob - a.sbase;
    for (int i = tid; i < s_pod.blob_len; i += 256) s_blob[i] = a.sprog[boff + i];
    gprog = a.sprog - a.sbase;   // the node set (outside the blob) is staged too (host-checked)
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      if (tid < (int)(sizeof(ksg_pod) / 4))
        reinterpret_cast<int32_t*>(a.wpods)[tid] = reinterpret_cast<const int32_t*>(&s_pod)[tid];
      for (int64_t i = tid; i < a.slen; i += 256) a.wprog[i] = a.sprog[i];
    }
  } else {
    stage_pod<256>(a.pods, a.prog, a.b0 + j, &s_pod, s_blob);
  }
  __syncthreads();
  const PodView v = make_view(c, s_prof, s_pod, s_blob, gprog, false, a.st.ports);
  const int n = blockIdx.x * 256 + tid;
  const size_t o = (size_t)(a.out0 + j);
  int32_t feas = 0, mt = 0, ma = 0, lo = 0;
  if (n < N) {
    NodeCols L;
    load_cols(c, a.st.requested, a.st.nonzero, a.st.pod_count, n, L);
    for (int k = j; k < a.nb; k++) {   // undo the pods placed on n at or after pod j's turn
      if (s_pl[k] != n) continue;
      const ksg_pod& q = a.pods[a.b0 + k];
#pragma unroll
      for (int r = 0; r < KSG_MAX_RES; r++)
        if (r < c.R) L.req[r] -= q.req[r];
      L.nz_cpu -= q.nz_cpu;
      L.nz_mem -= q.nz_mem;
      L.pod_count -= 1;
    }
    int64_t lraw[KSG_NPLUGINS] = {};
    const NodeEval e = eval_node_src(c, s_prof, v, GNode{&c, n}, L, n, nullptr, nullptr, nullptr, lraw);
    a.fstatus[o * NN + n] = e.st;
    a.rec[(size_t)j * NN + n] = pack_rec(e);
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
      cap_put(a.raw, (o * a.n_rows + q) * NN + n, x, a.narrow);
      // plugins without ScoreExtensions record the raw score again; the two
      // normalised ones are overwritten by ksg_capture_norm
      cap_put(a.norm, (o * a.n_rows + q) * NN + n,
              (pl == KSG_PL_TAINT_TOLERATION || pl == KSG_PL_NODE_AFFINITY) ? 0 : x, a.narrow);
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
  if (a.best) lo = (int32_t)wave_max64(lo);
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
    if (f) atomicAdd(&a.stats[4 * j], f);
    if (t) atomicMax(&a.stats[4 * j + 1], t);
    if (m) atomicMax(&a.stats[4 * j + 2], m);
    if (a.best && l) atomicMax(&a.stats[4 * j + 3], l);
  }
}
#endif  // KSG_PART

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_capture_norm(CapArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ unsigned long long s_key[4];
  __shared__ uint32_t s_err[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = blockIdx.y;
  const DevCluster& c = a.c;
  const int N = c.N;
  const size_t NN = N;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(a.prof)[i_];
  if (a.next && blockIdx.x == 0 && tid < 8) a.next[tid] = 0;   // the next call's slot
  stage_pod<256>(a.pods, a.prog, a.b0 + j, &s_pod, s_blob);
  __syncthreads();
  const PodView v = make_view(c, s_prof, s_pod, s_blob, a.prog, false, a.st.ports);
  const int n = blockIdx.x * 256 + tid;
  const int32_t nfeas = a.stats[4 * j], max_t = a.stats[4 * j + 1], max_a = a.stats[4 * j + 2];
  if (a.best) {   // selectHost over this block's nodes, merged by one atomic per block
    uint64_t key = 0;
    uint32_t err = 0;
    if (n < N && nfeas >= 2) {
      const uint64_t x = a.rec[(size_t)j * NN + n];
      if (x >> 63)
        key = argmax_key(total_score(v, (uint32_t)x, (x >> 48) & 0xff, (x >> 32) & 0xffff, max_t, max_a, err,
                                     nullptr, nullptr), n);
    }
    key = wave_max_u64(key);
    err = wave_or32(err);
    if (lane == 0) { s_key[wv] = key; s_err[wv] = err; }
    __syncthreads();
    if (tid == 0) {
      uint64_t k = 0;
      uint32_t e = 0;
      for (int i = 0; i < 4; i++) { k = s_key[i] > k ? s_key[i] : k; e |= s_err[i]; }
      if (k) atomicMax(a.best, (unsigned long long)k);
      if (e) atomicOr(a.err, e);
    }
  }
  if (n >= N) return;
  const size_t o = (size_t)(a.out0 + j);
  const uint64_t x = a.rec[(size_t)j * NN + n];
  int64_t total = 0, nt = 0, na = 0;
  if (nfeas >= 2 && (x >> 63)) {
    uint32_t err = 0;
    total = total_score(v, (uint32_t)x, (x >> 48) & 0xff, (x >> 32) & 0xffff, max_t, max_a, err, &nt, &na);
  }
  if (a.total) cap_put(a.total, o * NN + n, total, a.narrow);
  for (int q = 0; q < a.n_rows; q++) {
    const int pl = a.rows[q];
    if (nfeas < 2) {   // fewer than two feasible nodes: no Score runs, nothing recorded
      cap_put(a.raw, (o * a.n_rows + q) * NN + n, 0, a.narrow);
      cap_put(a.norm, (o * a.n_rows + q) * NN + n, 0, a.narrow);
    } else if (pl == KSG_PL_TAINT_TOLERATION) {
      cap_put(a.norm, (o * a.n_rows + q) * NN + n, nt, a.narrow);
    } else if (pl == KSG_PL_NODE_AFFINITY) {
      cap_put(a.norm, (o * a.n_rows + q) * NN + n, na, a.narrow);
    }
  }
}
#endif  // KSG_PART

