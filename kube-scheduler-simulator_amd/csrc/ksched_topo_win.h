// The speculative topology queue (configs[2]: PodTopologySpread /
// InterPodAffinity pods, one replica), included by ksched_dev.h after
// ksched_topo_coop.h.
//
// ksg_topo_coop walks the queue one pod at a time: three grid barriers per pod
// and every phase a latency chain (profiles/r5/stamps_topo_queue.txt).  Most
// consecutive pods do not read what the previous ones write, though.  A pod's
// assume changes (a) the resource columns of its node and (b) the topology
// counts of the selectors its labels match (cnt, the domain tables) and of the
// term templates it owns.  Pod j reads (b) only through the selectors of its
// spread constraints and affinity terms and through the templates matching
// its labels.  So when no earlier pod of a window writes what pod j reads
// (the host's window lengths, win_len), pod j at the window's start and pod j
// after the earlier window pods differ only at the nodes those pods took, and
// only in NodeResourcesFit / BalancedAllocation: the same one-changed-node
// premise as the configs[1] speculate-and-verify walk.
//
// Per window (up to kmax pods, device-driven: no host round trip per window):
//   ksg_topo_coop<1, LL, 3>  grid (G, kmax): row y runs pod first + y through
//                            the queue kernel's phases 1-3 against the
//                            window's start state (its own barrier flags
//                            among its G workgroups), then stores each node's
//                            static total (the weighted total less Fit and
//                            BalancedAllocation) and each tile's y + 1 best
//                            keys, and the pod's facts (WinPod)
//   walk_window              the last workgroup of those rows to finish, in
//                            the same launch: pod by pod, the changed nodes
//                            re-evaluated (Fit filter, Fit / BalancedAllocation
//                            scores on the current columns), the best
//                            unchanged node from the tiles' lists, selectHost;
//                            then every assume of the window (node columns,
//                            counts, domain tables, template tables) and the
//                            cursor advanced.
// A changed node a pod found feasible at the window's start and now fails
// NodeResourcesFit on ends the window before that pod (its normalisation
// extremes and feasible count may have moved): the next window starts there.
// The first pod of a window has no changed node, so every window decides at
// least one pod.  Results equal ksg_topo_coop's and the oracle's bit for bit.

constexpr int kWinMax = 8;   // pods per window (grid rows; G * kmax workgroups co-resident)

// A window pod's facts at the window's start (the rows store them, the walk
// reads them): what phase 4 would decide from, less the argmax.
struct WinPod {
  int32_t ok, nfeas, minidx, scored;
  uint32_t err;          // ScoreError bits of every workgroup (or-ed; the walk zeroes it)
  uint32_t status;       // KSG_ST_IPA_* flags
  uint32_t score_skip;
  uint32_t smask;        // the pod's Score plugins (make_view)
  int32_t w_fit, w_ba;
  int32_t fit_on;        // NodeResourcesFit's Filter runs for the pod
  int32_t pad;
};

struct WalkArgs {
  DevCluster c;
  DevState st;
  TopoTables tt;
  int32_t use_tables;
  int32_t* cursor;                    // the run's first undecided pod
  int32_t win_base, G, K;             // the run's first pod; tiles; the rows' list stride (kmax)
  const int32_t* win_tot;             // [kmax][N]
  const unsigned long long* win_top;  // [kmax][G][kmax]
  WinPod* win_pod;                    // [kmax]
  const int32_t* prog;                // the program pool (commit programs)
  int32_t* placements;                // [pods of the run]
  ksg_result* results;                // [pods of the run] or null
  unsigned long long* wstats;         // [0] windows, [1] pods decided, [2] windows ended by a changed node
};

// The walk keeps every node it touches in LDS: the columns the window's
// decisions changed (requested, non-zero, pod count: its own assumes, applied
// here) and the rows' static totals there.  Prefetched for each pod's best
// candidate (usually its decision), loaded on demand else.
struct WalkNode {
  int32_t node;
  NodeCols cols;
  int32_t wt[kWinMax];   // win_tot[i][node] of the window's pods
};
constexpr int kWalkNodes = 2 * kWinMax;

struct WalkLds {
  WinPod wp[kWinMax];
  unsigned long long cand[kWinMax][kWinMax];   // pod i's best i + 1 keys over every tile
  int ncand[kWinMax];
  WalkNode nodes[kWalkNodes];
  int nn;                                      // cache entries in use
  int chg[kWinMax];                            // the nodes the window's decided pods took
  int sel[kWinMax];                            // each decided pod's node (-1: none)
  unsigned long long ck[4];
  int drop;
};

// Threads f in [0, 32) of the workgroup load node n into e: its columns as the
// global state holds them (the window's earlier assumes never touched a node
// outside the cache) and its static totals; the caller synchronises.  The
// rows' outputs are read with agent-scope loads (stored with agent-scope
// stores by other workgroups of the launch).
__device__ __forceinline__ void walk_fetch(const WalkArgs& a, int len, int f, int n, WalkNode& e) {
  const DevCluster& c = a.c;
  const size_t N = c.N;
  const int R = c.R;
  if (f == 0) e.node = n;
  if (f < KSG_MAX_RES) {
    e.cols.alloc[f] = f < R ? c.alloc[f * N + n] : 0;
    e.cols.req[f] = f < R ? a.st.requested[f * N + n] : 0;
  } else if (f == KSG_MAX_RES) {
    e.cols.nz_cpu = a.st.nonzero[n];
  } else if (f == KSG_MAX_RES + 1) {
    e.cols.nz_mem = a.st.nonzero[N + n];
  } else if (f == KSG_MAX_RES + 2) {
    e.cols.pod_count = a.st.pod_count[n];
  } else if (f == KSG_MAX_RES + 3) {
    e.cols.allowed = c.allowed[n];
  } else if (f >= KSG_MAX_RES + 4 && f < KSG_MAX_RES + 4 + kWinMax) {
    const int i = f - (KSG_MAX_RES + 4);
    e.wt[i] = i < len ? gld(a.win_tot + (size_t)i * N + n) : -1;
  }
}

// The window [first, first + len) decided by one workgroup of 256 threads,
// pod by pod.  Everything a decision reads is in LDS after the prologue's two
// round trips (the facts and merged candidate lists, then the candidates'
// nodes), so a pod costs a few hundred cycles of LDS and wave reductions; the
// global assumes (atomics, fire and forget) are issued once the window is
// decided (no pod of the window reads the counts or tables another writes:
// the window lengths' premise).  pods: the window's records (LDS).
__device__ __forceinline__ void walk_window(const WalkArgs& a, int first, int len, const ksg_profile& prof,
                                            const ksg_pod* pods, WalkLds& L) {
  constexpr int NW = 4;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N, G = a.G, K = a.K;
  // ---- prologue: the facts; per pod (one wave each) its merged candidate
  // list, its i + 1 best keys over the G tiles' lists -------------------------
  constexpr int WW = (int)(sizeof(WinPod) / 4);
  for (int x = tid; x < len * WW; x += 256)
    reinterpret_cast<int32_t*>(L.wp)[x] = gld(reinterpret_cast<const int32_t*>(a.win_pod) + x);
  for (int i = wv; i < len; i += NW) {
    const int kk = i + 1, total = G * kk;
    unsigned long long v[8];   // the lane's best 8 entries (t, r), r < kk, of tile t's list
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int x = lane + 64 * u, t = x / kk, r = x - t * kk;
      v[u] = x < total ? gld(a.win_top + ((size_t)i * G + t) * K + r) : 0ull;
    }
    for (int x = lane + 8 * 64; x < total; x += 64) {   // (more entries: keep the lane's best 8)
      const int t = x / kk, r = x - t * kk;
      unsigned long long y = gld(a.win_top + ((size_t)i * G + t) * K + r);
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (y > v[u]) { const unsigned long long z = v[u]; v[u] = y; y = z; }
    }
    int nc = 0;
    for (int r = 0; r < kk; r++) {
      unsigned long long m = 0;
#pragma unroll
      for (int u = 0; u < 8; u++) m = v[u] > m ? v[u] : m;
      m = wreduce(m, OpMaxU64{});
      if (!m) break;
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (v[u] == m) v[u] = 0;
      if (lane == 0) L.cand[i][r] = m;
      nc++;
    }
    if (lane == 0) L.ncand[i] = nc;
  }
  __syncthreads();
  {   // pod q's best candidate into entry q (duplicates allowed: lookups and
      // assumes use the first entry holding a node)
    const int q = tid >> 5, f = tid & 31;
    if (q < len) {
      const int n = L.ncand[q] ? key_node(L.cand[q][0]) : -1;
      if (n >= 0) walk_fetch(a, len, f, n, L.nodes[q]);
      else if (f == 0) L.nodes[q].node = -1;
    }
    if (tid == 0) L.nn = len;
  }
  __syncthreads();
  const CmProf cm = cm_prof(prof);
  int n_chg = 0, decided = 0;
  bool cut = false;
  auto entry_of = [&](int n) {
    int e = -1;
    for (int q = L.nn - 1; q >= 0; q--) e = L.nodes[q].node == n ? q : e;
    return e;
  };
  for (int i = 0; i < len; i++) {
    const ksg_pod& p = pods[i];
    const WinPod& wp = L.wp[i];
    const int ok = wp.ok, nfeas = wp.nfeas, scored = wp.scored;
    // wave 0: the changed nodes against their columns now; wave 1: the best
    // candidate outside the changed set (lane r: candidate r)
    uint64_t k = 0;
    int drop = 0;
    if (wv == 0 && lane < n_chg && ok) {
      const int m = L.chg[lane];
      const WalkNode& e = L.nodes[entry_of(m)];
      const int32_t w = e.wt[i];
      if (w >= 0) {
        const NodeCols& C = e.cols;
        if (wp.fit_on && fit_filter(c, p, C, prof.fit_ignored_res)) {
          drop = 1;
        } else if (scored) {
          int64_t part = 0;
          const uint32_t sm = wp.smask;
          if (cm.fast && (sm & (bit(KSG_PL_NODE_RESOURCES_FIT) | bit(KSG_PL_BALANCED_ALLOCATION)))) {
            int64_t sf, sb;
            fit_ba_cm(cm, p, C, sf, sb);
            if (sm & bit(KSG_PL_NODE_RESOURCES_FIT)) part += sf * wp.w_fit;
            if (sm & bit(KSG_PL_BALANCED_ALLOCATION)) part += sb * wp.w_ba;
          } else {
            if (sm & bit(KSG_PL_NODE_RESOURCES_FIT)) part += fit_score(prof, p, C) * wp.w_fit;
            if (sm & bit(KSG_PL_BALANCED_ALLOCATION)) part += ba_score(prof, p, C) * wp.w_ba;
          }
          k = argmax_key((int64_t)w + part, m);
        }
      }
    } else if (wv == 1 && ok && scored) {
      const unsigned long long x = lane < L.ncand[i] ? L.cand[i][lane] : 0ull;
      bool in = false;
      const int n = key_node(x);
      for (int q = 0; q < n_chg; q++) in |= L.chg[q] == n;
      const unsigned long long b = __ballot(x != 0 && !in);
      if (b) k = __shfl(x, __builtin_ctzll(b));
    }
    k = wreduce(k, OpMaxU64{});
    drop = __any(drop) ? 1 : 0;
    if (lane == 0) L.ck[wv] = k;
    if (tid == 0) L.drop = 0;
    __syncthreads();
    if (lane == 0 && wv == 0 && drop) L.drop = 1;
    __syncthreads();
    if (L.drop) {   // a changed node left the pod's feasible set: the window ends before it
      cut = true;
      break;
    }
    int selected = -1;
    uint32_t status = wp.status;
    if (!ok) {
      status |= KSG_ST_SCORE_ERROR;
    } else if (nfeas == 1) {
      selected = wp.minidx;
    } else if (scored) {
      status |= KSG_ST_SCORED;
      const unsigned long long b = L.ck[0] > L.ck[1] ? L.ck[0] : L.ck[1];
      if (wp.err & 1u) status |= KSG_ST_SCORE_ERROR;
      else selected = b ? key_node(b) : -1;
    }
    if (selected >= 0 && entry_of(selected) < 0) {   // not cached: its columns and static totals now
      if (tid < 32) walk_fetch(a, len, tid, selected, L.nodes[L.nn]);
      __syncthreads();
      if (tid == 0) L.nn++;
      __syncthreads();
    }
    if (tid == 0) {
      if (selected >= 0) {   // the assume on the cached columns (globally after the window)
        NodeCols& C = L.nodes[entry_of(selected)].cols;
        for (int r = 0; r < c.R; r++) C.req[r] += p.req[r];
        C.nz_cpu += p.nz_cpu;
        C.nz_mem += p.nz_mem;
        C.pod_count += 1;
        L.chg[n_chg] = selected;
      }
      L.sel[i] = selected;
      a.placements[first + i - a.win_base] = selected;
      if (a.results) {
        ksg_result res;
        res.selected = selected;
        res.n_feasible = nfeas;
        res.status = status;
        res.score_skip = wp.score_skip;
        a.results[first + i - a.win_base] = res;
      }
    }
    if (selected >= 0) n_chg++;
    decided++;
    __syncthreads();
  }
  // ---- the window's assumes in global memory, every pod at once (wave w:
  // pods w, w + 4, ..; lane 0 the resource columns, the other lanes the
  // matched selectors (count, domain tables, count-of-counts) and the owned
  // templates) ---------------------------------------------------------------
  const DevState& st = a.st;
  const size_t NN = N;
  for (int i = wv; i < decided; i += NW) {
    const int n = L.sel[i];
    if (n < 0) continue;
    const ksg_pod& p = pods[i];
    if (lane == 0) {
      for (int r = 0; r < c.R; r++)
        __hip_atomic_fetch_add((__attribute__((address_space(1))) int64_t*)(st.requested + r * NN + n), p.req[r],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((__attribute__((address_space(1))) int64_t*)(st.nonzero + n), p.nz_cpu, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((__attribute__((address_space(1))) int64_t*)(st.nonzero + NN + n), p.nz_mem,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gadd(st.pod_count + n, 1);
    }
    if (p.commit < 0) continue;
    const int32_t* cprog = a.prog + p.commit;
    const int ns = cprog[0];
    const int32_t* tw = cprog + 1 + ns;
    const int nt = tw[0];
    for (int q = lane; q < ns + nt; q += 64) {
      if (q < ns) {   // selector s: its count at n (the old value moves the count-of-counts), its tables
        const int s = cprog[1 + q];
        const int32_t old = __hip_atomic_fetch_add(
            (__attribute__((address_space(1))) int32_t*)(st.cnt + (size_t)s * NN + n), 1, __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        if (a.use_tables) {
          const TopoTables& t = a.tt;
          for (int e = t.sp_off[s]; e < t.sp_off[s + 1]; e++) {
            const uint32_t v = c.label_val[(size_t)t.sp[2 * e] * NN + n];
            if (v) gadd(t.dom + t.sp[2 * e + 1] + v, 1);
          }
          gadd(t.tot + s, 1);
          const int co = t.cc_off[s];
          if (co >= 0) {
            if (old + 1 >= t.Kc - 1) {
              gst(t.invalid, 1u);
            } else {
              gadd(t.cc + co + old, -1);
              gadd(t.cc + co + old + 1, 1);
            }
          }
        }
      } else {   // an owned term template: its domain entry and total
        const int x = q - ns, tm = tw[1 + 2 * x];
        const uint32_t val = c.label_val[(size_t)c.tmpl_col[tm] * NN + n];
        if (!val) continue;
        gadd(st.tab + c.tmpl_off[tm] + val, c.tmpl_kind[tm] == KSG_TMPL_PREF ? tw[2 + 2 * x] : 1);
        gadd(st.tmpl_total + tm, 1);
      }
    }
  }
  for (int i = tid; i < len; i += 256) gst(&a.win_pod[i].err, 0u);   // (the next window's rows or into it)
  if (tid == 0) {
    gst(a.cursor, first + decided);
    if (a.wstats) {
      atomicAdd(&a.wstats[0], 1ull);
      atomicAdd(&a.wstats[1], (unsigned long long)decided);
      if (cut) atomicAdd(&a.wstats[2], 1ull);
    }
  }
}
