// Single-replica queue with PodTopologySpread / InterPodAffinity across the
// whole chip (config 3), included by ksched.hip inside its anonymous namespace.
//
// ksg_queue_topo_kernel walks every node of a pod four times from ONE
// workgroup; at 15,000 nodes that is ~30 dependent node visits per lane per
// sweep, 1.2 ms per pod.  Here G co-resident workgroups share each pod: lane
// (wg, tid) owns nodes (k * G + wg) * 256 + tid, k < KN, for the whole queue,
// so a node's mutable columns (requested, non-zero, pod count, selector
// counts) are only ever read and written by one lane.  Per pod:
//
//   setup      every workgroup stages the pod and lays out its LDS histograms
//   phase 1    pre-pass over the lane's nodes: per-domain counts into the LDS
//              histograms, merged into a global accumulator set (atomics)
//   -- grid barrier --
//   phase 2    every workgroup copies the merged histograms back into LDS;
//              sweep A (filters incl. PTS/IPA, node-local scores), the IPA raw
//              score and, with one soft PTS constraint, the extremes of its
//              per-node count; reductions into the accumulator set
//   -- grid barrier --  (+ one more for >= 2 soft PTS constraints: their raw
//                         scores' min/max)
//   phase 3    normalise, weight, argmax; atomicMax of the packed key
//   -- grid barrier --
//   phase 4    every workgroup reads the selection; the owner lane of the
//              selected node assumes the pod (node columns, selector counts;
//              domain tables by atomics)
//
// With one soft constraint the PodTopologySpread raw score of a node is
// round(m * w + maxSkew - 1) for a node with the topology key (0 without it),
// m its domain count and w = log(size + 2) > 0, which is monotone in m: the
// min / max over the feasible nodes follow from the min / max of m, so the
// sizes and the min / max need no extra barrier.
//
// Accumulator sets alternate by pod parity; workgroup 0 resets the set of pod
// j - 1 in phase 2 of pod j (every workgroup has read it by then).  Grid
// barrier: a monotonic arrival counter; every storing wave drains its stores,
// one lane releases (agent scope), arrives, polls relaxed with s_sleep, and
// acquires (agent scope); every cross-workgroup word is read with agent-scope
// atomic loads (MI355X guide, Guideline 16).  The poll is bounded: on timeout
// the kernel records an error and every workgroup leaves.

struct CoopAcc {
  // phase 1
  unsigned long long hard_min[kMaxHard];   // order-preserving encoding (enc64)
  int32_t hard_dom[kMaxHard];
  long long soft_empty[kMaxSoft];
  long long aff_total;
  int32_t pref_any;
  // phase 2
  int32_t nfeas;
  int32_t minidx;                           // atomicMin
  int32_t soft_present[kMaxSoft], soft_empty_seen[kMaxSoft], n_ignored;
  int32_t has_val, has_zero, err;
  unsigned long long max_t, max_a;          // atomicMax (non-negative)
  unsigned long long mmin, mmax;            // one soft constraint: extremes of m (enc64)
  unsigned long long imin, imax;            // IPA raw extremes (enc64)
  unsigned long long pmin, pmax;            // >= 2 soft constraints: raw extremes (enc64)
  // phase 3
  unsigned long long best;
  int32_t hist[KSG_HIST_MAX];               // merged LDS histograms (counts added, bitmaps or-ed)
};

__device__ __forceinline__ unsigned long long enc64(long long x) { return (unsigned long long)x ^ (1ull << 63); }
__device__ __forceinline__ long long dec64(unsigned long long x) { return (long long)(x ^ (1ull << 63)); }

template <class T>
__device__ __forceinline__ T ald(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void coop_acc_init(CoopAcc* a, int words) {
  // called by one workgroup; plain stores, published by the next grid barrier
  const int tid = threadIdx.x;
  if (tid == 0) {
    for (int i = 0; i < kMaxHard; i++) { a->hard_min[i] = enc64(0x7fffffffffffffffll); a->hard_dom[i] = 0; }
    for (int i = 0; i < kMaxSoft; i++) { a->soft_empty[i] = 0; a->soft_present[i] = 0; a->soft_empty_seen[i] = 0; }
    a->aff_total = 0;
    a->pref_any = 0;
    a->nfeas = 0;
    a->minidx = 0x7fffffff;
    a->n_ignored = 0;
    a->has_val = a->has_zero = a->err = 0;
    a->max_t = a->max_a = 0;
    a->mmin = a->imin = a->pmin = enc64(0x7fffffffffffffffll);
    a->mmax = a->imax = a->pmax = enc64(-0x7fffffffffffffffll - 1);
    a->best = 0;
  }
  for (int i = tid; i < words; i += blockDim.x) a->hist[i] = 0;
}

__global__ void ksg_topo_coop_init(CoopAcc* acc) {
  coop_acc_init(acc + blockIdx.x, KSG_HIST_MAX);
}

struct CoopArgs {
  DevCluster c;
  DevState st;
  const ksg_pod* pods;
  const int32_t* prog;
  const ksg_profile* profile;
  int32_t first, count, G;
  int32_t* placements;
  ksg_result* results;      // or null
  CoopAcc* acc;             // [2]
  unsigned* bar;            // arrival counter, zeroed before the launch
  unsigned* timeout;        // set when a barrier poll gave up
};

__device__ __forceinline__ bool coop_barrier(const CoopArgs& a, unsigned& target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  target += (unsigned)a.G;
  __shared__ int s_timeout;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(a.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int to = 0;
    while (__hip_atomic_load(a.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 25) ||
          __hip_atomic_load(a.timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(a.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        to = 1;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_timeout = to;
  }
  __syncthreads();
  return s_timeout == 0;
}

// PodTopologySpread with one soft constraint: the per-node count m of
// pts_score_node (same branches), or ignored / no key.  0: m valid, 1: the
// node lacks the key (score 0), 2: ignored node (score -1).
__device__ __forceinline__ int pts_soft1_m(const DevCluster& c, const PodView& v, const TopoCtx& t, int n,
                                          int64_t& m) {
  const TopoProg& g = *t.g;
  const TopoShared& s = *t.s;
  if (g.require_all && !has_all(c, g.soft, g.n_soft, 6, n)) return 2;
  const int32_t* sc = g.soft;
  const uint32_t val = lab(c, sc[0], n);
  if (!val) return 1;
  const Slot& sl = s.soft[0];
  if (sc[5]) m = cnt_at(t.cnt, c.N, sl.sel, n);
  else if (!sl.unique) m = t.hist[sl.hist + val];
  else if (val == 1) m = s.soft_empty[0];
  else m = inclusion(c, v, sc[3], sc[4], n) ? cnt_at(t.cnt, c.N, sl.sel, n) : 0;
  return 0;
}

__device__ __forceinline__ int64_t pts_soft1_score(const TopoProg& g, const TopoShared& s, int64_t m) {
  const double x = (double)m * s.soft_w[0];
  double score = 0.0;
  score += x + (double)(g.soft[2] - 1);
  return (int64_t)round(score);
}

// NodeInfo.AddPod for node n by the lane that owns it: node columns and
// selector counts with plain stores, domain tables with atomics.
__device__ void coop_commit(const DevCluster& c, const DevState& st, const ksg_pod& p, const int32_t* commit_prog,
                            int n) {
  const int N = c.N;
  for (int r = 0; r < c.R; r++) st.requested[(size_t)r * N + n] += p.req[r];
  st.nonzero[n] += p.nz_cpu;
  st.nonzero[(size_t)N + n] += p.nz_mem;
  st.pod_count[n] += 1;
  if (commit_prog) {
    const int32_t* w = commit_prog;
    const int ns = *w++;
    for (int i = 0; i < ns; i++) st.cnt[(size_t)w[i] * N + n] += 1;
    w += ns;
    const int nt = *w++;
    for (int i = 0; i < nt; i++) {
      const int t = w[i];
      const uint32_t val = c.label_val[(size_t)c.tmpl_col[t] * N + n];
      if (!val) continue;
      __hip_atomic_fetch_add(st.tab + c.tmpl_off[t] + val, c.tmpl_kind[t] == KSG_TMPL_PREF ? c.tmpl_weight[t] : 1,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(st.tmpl_total + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int KN>
__global__ __launch_bounds__(256) void ksg_topo_coop(CoopArgs a) {
  constexpr int BLOCK = 256, NW = BLOCK / 64;
  constexpr long long BIG = 0x7fffffffffffffffll;
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ __attribute__((aligned(16))) int32_t s_hist[KSG_HIST_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ TopoProg s_g;
  __shared__ TopoShared s_t;
  __shared__ long long s_r[NW][8];
  __shared__ int s_size[kMaxSoft];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wg = blockIdx.x, G = a.G;
  const DevCluster& c = a.c;
  const int N = c.N;
  const DevState& st = a.st;
  if (tid < (int)(sizeof(ksg_profile) / 4))
    reinterpret_cast<int32_t*>(&s_prof)[tid] = reinterpret_cast<const int32_t*>(a.profile)[tid];
  __syncthreads();
  const ksg_profile& prof = s_prof;
  bool ipa_in_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_in_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  const bool ipa_in_score = (prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u;
  unsigned target = 0;
  int prev_words = KSG_HIST_MAX;

  auto node_of = [&](int k) { return (k * G + wg) * BLOCK + tid; };

  for (int kq = 0; kq < a.count; kq++) {
    const int pi = a.first + kq;
    CoopAcc* acc = a.acc + (kq & 1);
    CoopAcc* nxt = a.acc + ((kq + 1) & 1);
    __syncthreads();
    stage_pod<BLOCK>(a.pods, a.prog, pi, &s_pod, s_blob);
    __syncthreads();
    const ksg_pod& p = s_pod;
    if (tid == 0) {
      const PodView v0 = make_view(c, prof, p, s_blob, a.prog, true);
      parse_topo(p, s_blob, v0.fskip, v0.smask, s_g);
      layout_slots(c, s_g, s_t);
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
    const int words = ok ? s_t.words : 0;
    for (int i = tid; i < words; i += BLOCK) s_hist[i] = 0;
    PodView v = make_view(c, prof, p, s_blob, a.prog, true);
    const TopoProg& g = s_g;
    const TopoCtx tc{&s_g, &s_t, s_hist, st.cnt, st.tab, true};
    __syncthreads();

    // ---- phase 1: pre-pass over this lane's nodes -------------------------
    const bool pre = ok && (g.pts_filter || g.pts_score || g.ipa);
    if (pre) {
      long long lmin[kMaxHard], ldom[kMaxHard], lempty[kMaxSoft], laff = 0, lany = 0;
      for (int i = 0; i < kMaxHard; i++) { lmin[i] = BIG; ldom[i] = 0; }
      for (int i = 0; i < kMaxSoft; i++) lempty[i] = 0;
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N) break;
        if (g.pts_filter && has_all(c, g.hard, g.n_hard, 7, n)) {
          for (int i = 0; i < g.n_hard; i++) {
            const int32_t* h = g.hard + 7 * i;
            if (!inclusion(c, v, h[5], h[6], n)) continue;
            const Slot& sl = s_t.hard[i];
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
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
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
            if (sl.unique) {
              if (val == 1) lempty[i] += x;
            } else {
              atomicAdd(&s_hist[sl.hist + val], x);
            }
          }
        }
        if (g.ipa) {
          if (g.n_aff > 0) {
            const int32_t x = cnt_at(st.cnt, N, g.sel_all, n);
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
            atomicAdd(&s_hist[sl.hist + val], cnt_at(st.cnt, N, sl.sel, n));
            atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
          }
          for (int i = 0; i < g.n_pref; i++) {
            const Slot& sl = s_t.pref[i];
            const uint32_t val = lab(c, sl.col, n);
            if (!val) continue;
            const int32_t x = cnt_at(st.cnt, N, sl.sel, n);
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
      // merge this workgroup's part into the pod's accumulator set
      auto merge_slot = [&](const Slot& sl) {
        if (sl.unique) return;
        for (int i = tid; i < sl.V; i += BLOCK)
          if (s_hist[sl.hist + i]) atomicAdd(&acc->hist[sl.hist + i], s_hist[sl.hist + i]);
        const int bw = (sl.V + 31) / 32;
        for (int i = tid; i < bw; i += BLOCK)
          if (s_hist[sl.pres + i]) atomicOr((uint32_t*)&acc->hist[sl.pres + i], (uint32_t)s_hist[sl.pres + i]);
      };
      for (int i = 0; i < g.n_hard; i++) merge_slot(s_t.hard[i]);
      for (int i = 0; i < g.n_soft; i++) merge_slot(s_t.soft[i]);
      for (int i = 0; i < g.n_aff; i++) merge_slot(s_t.aff[i]);
      for (int i = 0; i < g.n_anti; i++) merge_slot(s_t.anti[i]);
      for (int i = 0; i < g.n_pref; i++) merge_slot(s_t.pref[i]);
      if (tid == 0) {
        for (int i = 0; i < g.n_hard; i++)
          if (s_t.hard[i].unique) {
            if (s_t.hard_dom[i]) atomicMin(&acc->hard_min[i], enc64(s_t.hard_min[i]));
            if (s_t.hard_dom[i]) atomicAdd(&acc->hard_dom[i], s_t.hard_dom[i]);
          }
        for (int i = 0; i < g.n_soft; i++)
          if (s_t.soft_empty[i]) atomicAdd((unsigned long long*)&acc->soft_empty[i], (unsigned long long)s_t.soft_empty[i]);
        if (s_t.aff_total) atomicAdd((unsigned long long*)&acc->aff_total, (unsigned long long)s_t.aff_total);
        if (s_t.pref_any) atomicOr(&acc->pref_any, 1);
      }
    }
    if (!coop_barrier(a, target)) return;

    // ---- phase 2: merged counts back into LDS; sweep A ----------------------
    if (pre) {
      for (int i = tid; i < words; i += BLOCK) s_hist[i] = ald(&acc->hist[i]);
      if (tid == 0) {
        for (int i = 0; i < g.n_hard; i++)
          if (s_t.hard[i].unique) {
            s_t.hard_min[i] = dec64(ald(&acc->hard_min[i]));
            s_t.hard_dom[i] = ald(&acc->hard_dom[i]);
          }
        for (int i = 0; i < g.n_soft; i++) s_t.soft_empty[i] = ald(&acc->soft_empty[i]);
        s_t.aff_total = ald(&acc->aff_total);
        s_t.pref_any = ald(&acc->pref_any);
      }
      __syncthreads();
      for (int i = 0; i < g.n_hard; i++) {   // minimum over present domains of the non-unique hard slots
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
    }
    if (wg == 0) coop_acc_init(nxt, prev_words);   // the set of pod kq - 1, read by everyone by now
    prev_words = words;
    __syncthreads();
    if (tid == 0) {
      long long ma = 0, mh = 0, mp = 0;
      for (int i = 0; i < g.n_ma; i++) ma += ald(&st.tmpl_total[g.m_anti[i]]);
      for (int i = 0; i < g.n_mh; i++) mh += ald(&st.tmpl_total[g.m_hard[i]]);
      for (int i = 0; i < g.n_mp; i++) mp += ald(&st.tmpl_total[g.m_pref[i]]);
      s_t.ipa_skip_filter = !g.ipa || (ma == 0 && g.n_aff == 0 && g.n_anti == 0);
      s_t.ipa_skip_score = !g.ipa || !((prof.hard_pod_affinity_weight > 0 && mh > 0) || mp > 0);
      if (pre) {
        for (int i = 0; i < g.n_hard; i++)   // minMatchNum: 0 when fewer domains than minDomains
          if (s_t.hard_dom[i] < g.hard[7 * i + 3]) s_t.hard_min[i] = 0;
        if (s_t.pref_any) s_t.ipa_skip_score = 0;
      }
    }
    __syncthreads();
    if (s_t.ipa_skip_filter) v.fskip |= bit(KSG_PL_INTER_POD_AFFINITY);
    const bool ipa_may_score = ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
                               !s_t.ipa_skip_score;
    const bool soft1 = g.pts_score && g.n_soft == 1;

    NodeEval ev[KN];
    int64_t yv[KN];
    int32_t nfeas = 0, minidx = 0x7fffffff, lign = 0, has_val = 0, has_zero = 0;
    int64_t max_t = 0, max_a = 0;
    long long mmin = BIG, mmax = -BIG - 1, imin = BIG, imax = -BIG - 1;
    int lpres[kMaxSoft] = {0, 0, 0, 0}, lseen[kMaxSoft] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < KN; k++) {
      const int n = node_of(k);
      ev[k].st = 1;
      yv[k] = 0;
      if (n >= N || !ok) continue;
      ev[k] = eval_node(c, prof, v, st.requested, st.nonzero, st.pod_count, n, nullptr, nullptr, &tc);
      if (ev[k].st != 0) continue;
      nfeas += 1;
      minidx = min(minidx, n);
      max_t = max(max_t, ev[k].rt);
      max_a = max(max_a, ev[k].ra);
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
        if (soft1) {
          int64_t m = 0;
          const int r = pts_soft1_m(c, v, tc, n, m);
          if (r == 0) { has_val = 1; mmin = min(mmin, (long long)m); mmax = max(mmax, (long long)m); }
          else if (r == 1) has_zero = 1;
        }
      }
      if (ipa_may_score) {
        yv[k] = ipa_score_node(c, prof, tc, n);
        imin = min(imin, (long long)yv[k]);
        imax = max(imax, (long long)yv[k]);
      }
    }
    {
      nfeas = wave_sum32(nfeas);
      minidx = wave_min32(minidx);
      max_t = wave_max64(max_t);
      max_a = wave_max64(max_a);
      lign = wave_sum32(lign);
      has_val = wave_sum32(has_val);
      has_zero = wave_sum32(has_zero);
      mmin = wave_min64(mmin); mmax = wave_max64(mmax);
      imin = wave_min64(imin); imax = wave_max64(imax);
      if (lane == 0) {
        if (nfeas) {
          atomicAdd(&acc->nfeas, nfeas);
          atomicMin(&acc->minidx, minidx);
          atomicMax(&acc->max_t, (unsigned long long)max_t);
          atomicMax(&acc->max_a, (unsigned long long)max_a);
        }
        if (lign) atomicAdd(&acc->n_ignored, lign);
        if (has_val) {
          atomicOr(&acc->has_val, 1);
          atomicMin(&acc->mmin, enc64(mmin));
          atomicMax(&acc->mmax, enc64(mmax));
        }
        if (has_zero) atomicOr(&acc->has_zero, 1);
        if (imin <= imax) {
          atomicMin(&acc->imin, enc64(imin));
          atomicMax(&acc->imax, enc64(imax));
        }
      }
      if (g.pts_score) {
        for (int i = 0; i < g.n_soft; i++) {
          const int pr = wave_sum32(lpres[i]), se = (int)wave_or32((uint32_t)lseen[i]);
          if (lane == 0) {
            if (pr) atomicAdd(&acc->soft_present[i], pr);
            if (se) atomicOr(&acc->soft_empty_seen[i], 1);
          }
        }
      }
    }
    __syncthreads();
    if (g.pts_score && ok)   // domains seen among feasible nodes (non-unique soft slots)
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        for (int wd = tid; wd < (sl.V + 31) / 32; wd += BLOCK)
          if (s_hist[sl.mark + wd]) atomicOr((uint32_t*)&acc->hist[sl.mark + wd], (uint32_t)s_hist[sl.mark + wd]);
      }
    if (!coop_barrier(a, target)) return;

    // ---- phase 3: sizes, normalisation, argmax --------------------------------
    const int gnfeas = ald(&acc->nfeas);
    const bool scored = ok && gnfeas >= 2;
    const bool do_pts = scored && g.pts_score;
    const bool do_ipa = scored && ipa_may_score;
    long long pmin = BIG, pmax = 0, gimin = BIG, gimax = -BIG - 1;
    if (do_pts) {
      for (int i = 0; i < g.n_soft; i++) {
        const Slot& sl = s_t.soft[i];
        if (g.soft[6 * i + 5] || sl.unique) continue;
        int bits = 0;
        for (int wd = tid; wd < (sl.V + 31) / 32; wd += BLOCK) bits += __popc(ald((uint32_t*)&acc->hist[sl.mark + wd]));
        bits = wave_sum32(bits);
        if (lane == 0 && bits) atomicAdd(&s_size[i], bits);
      }
      __syncthreads();
      if (tid == 0) {
        const int n_ign = ald(&acc->n_ignored);
        for (int i = 0; i < g.n_soft; i++) {
          const Slot& sl = s_t.soft[i];
          int sz;
          if (g.soft[6 * i + 5]) sz = gnfeas - n_ign;
          else if (sl.unique) sz = ald(&acc->soft_present[i]) + ald(&acc->soft_empty_seen[i]);
          else sz = s_size[i];
          s_t.soft_w[i] = c.log_table[sz + 2];   // topologyNormalizingWeight = math.Log(size + 2)
        }
        long long lo = BIG, hi = 0;
        if (soft1) {
          if (ald(&acc->has_val)) {
            lo = pts_soft1_score(g, s_t, dec64(ald(&acc->mmin)));
            hi = pts_soft1_score(g, s_t, dec64(ald(&acc->mmax)));
          }
          if (ald(&acc->has_zero)) { lo = min(lo, 0ll); hi = max(hi, 0ll); }
        }
        s_r[0][0] = lo;
        s_r[0][1] = hi;
      }
      __syncthreads();
      pmin = s_r[0][0];
      pmax = s_r[0][1];
      if (!soft1) {   // >= 2 soft constraints: raw scores first, then their extremes
        long long lo = BIG, hi = 0;
#pragma unroll
        for (int k = 0; k < KN; k++) {
          const int n = node_of(k);
          if (n >= N || ev[k].st != 0) continue;
          const int64_t x = pts_score_node(c, v, tc, n);
          if (x >= 0) { lo = min(lo, (long long)x); hi = max(hi, (long long)x); }
        }
        lo = wave_min64(lo);
        hi = wave_max64(hi);
        if (lane == 0 && lo <= hi) {
          atomicMin(&acc->pmin, enc64(lo));
          atomicMax(&acc->pmax, enc64(hi));
        }
        if (!coop_barrier(a, target)) return;
        const long long l2 = dec64(ald(&acc->pmin)), h2 = dec64(ald(&acc->pmax));
        pmin = l2;
        pmax = l2 <= h2 ? h2 : 0;
      }
    }
    if (do_ipa) {
      gimin = dec64(ald(&acc->imin));
      gimax = dec64(ald(&acc->imax));
    }
    const int64_t gmax_t = (int64_t)ald(&acc->max_t), gmax_a = (int64_t)ald(&acc->max_a);
    if (scored) {
      uint64_t best = 0;
      uint32_t err = 0;
      const int64_t w_pts = prof.weight[KSG_PL_POD_TOPOLOGY_SPREAD], w_ipa = prof.weight[KSG_PL_INTER_POD_AFFINITY];
#pragma unroll
      for (int k = 0; k < KN; k++) {
        const int n = node_of(k);
        if (n >= N || ev[k].st != 0) continue;
        int64_t total = total_score(v, ev[k].part, ev[k].rt, ev[k].ra, gmax_t, gmax_a, err, nullptr, nullptr);
        if (do_pts) {   // PodTopologySpread.NormalizeScore
          const int64_t x = pts_score_node(c, v, tc, n);
          int64_t s;
          if (x < 0) s = 0;
          else if (pmax == 0) s = 100;
          else s = div_nonneg(100 * (pmax + pmin - x), pmax);
          err |= (s < 0 || s > 100);
          total += s * w_pts;
        }
        if (do_ipa) {   // InterPodAffinity.NormalizeScore (float64 min-max)
          const int64_t y = yv[k];
          const int64_t diff = gimax - gimin;
          double f = 0;
          if (diff > 0) f = (double)100 * ((double)(y - gimin) / (double)diff);
          const int64_t s = (int64_t)f;
          err |= (s < 0 || s > 100);
          total += s * w_ipa;
        }
        const uint64_t key = argmax_key(total, n);
        best = key > best ? key : best;
      }
      best = wave_max_u64(best);
      err = wave_or32(err);
      if (lane == 0) {
        if (best) atomicMax(&acc->best, (unsigned long long)best);
        if (err) atomicOr(&acc->err, 1);
      }
    }
    if (!coop_barrier(a, target)) return;

    // ---- phase 4: select and assume --------------------------------------------
    int selected = -1;
    uint32_t status = 0;
    if (!ok) {
      status |= KSG_ST_SCORE_ERROR;
    } else if (gnfeas == 1) {
      selected = ald(&acc->minidx);
    } else if (scored) {
      status |= KSG_ST_SCORED;
      if (ald(&acc->err)) status |= KSG_ST_SCORE_ERROR;
      else selected = key_node(ald(&acc->best));
    }
    if (selected >= 0 && ((selected / BLOCK) % G) == wg && (selected % BLOCK) == tid)
      coop_commit(c, st, p, p.commit >= 0 ? s_blob + (p.commit - p.blob) : nullptr, selected);
    if (wg == 0 && tid == 0) {
      uint32_t score_skip = p.score_skip;
      if (ipa_in_filter && s_t.ipa_skip_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
      if (scored && ipa_in_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u) && s_t.ipa_skip_score) {
        status |= KSG_ST_IPA_PRESCORE_SKIP;
        score_skip |= bit(KSG_PL_INTER_POD_AFFINITY);
      }
      a.placements[kq] = selected;
      if (a.results) {
        ksg_result res;
        res.selected = selected;
        res.n_feasible = ok ? gnfeas : 0;
        res.status = status;
        res.score_skip = score_skip;
        a.results[kq] = res;
      }
    }
  }
}
