// Phase 2, pipelined variant (KSG_BATCH_MODE=pipe, default): the per-pod
// critical chain holds the decision only.  Included by ksched.hip.
//
// Setting.  A batch of pods is walked in queue order against the changed set
// C (nodes assumed onto earlier in the batch, plus -- with the two-batch
// window -- the nodes the previous batch changed, whose phase-1 records were
// computed on an older state).  Pod j's choice is the best of (a) the best
// unchanged node bu_j, the first entry of the sorted top set T_j outside C,
// whose phase-1 key is exact, and (b) the changed nodes re-evaluated on their
// live columns.  Assuming pod j changes exactly one node.
//
// Pipelining.  For pod j + 1 the live key of changed slot s is one of two
// values: eval(pod j+1, row_s) if pod j goes elsewhere, eval(pod j+1, row_s +
// pod j) if pod j lands on s.  Neither depends on pod j's decision, so both
// are computed DURING step j, by two lanes per slot:
//   lanes [0, SLOTS)          version N: row_s
//   lanes [SLOTS, 2 SLOTS)    version C: row_s + pod j's request
// and the lane of the next free slot (version C) evaluates pod j + 1 on
// bu_j + pod j (the new slot pod j creates when it takes bu_j).  When pod j is
// decided, exactly one version per slot contributes to pod j + 1's reductions
// (max key, feasible / live / lost-holder counts), which are folded at the
// start of step j + 1.  Per step: fold, decide, mask, one wave reduction,
// one barrier; the evaluations overlap the decision.
//
// Prefetch.  At step j the top set T_{j+1} (in registers since step j - 1) is
// flagged against C; its first two unflagged entries are the candidates for
// bu_{j+1} (bu_{j+1} is the first of them that is not pod j's node), and
// their columns and phase-1 records go to an LDS candidate buffer, consumed
// at step j + 1.  Every slot lane keeps its node's records two pods ahead.
//
// Exactness.  Every value is the sequential one: version selection is exact
// by construction; a renormalisation (a phase-1 maximum whose every holder
// became infeasible) or a range error takes the full rescan of pod j's
// records with live maxima (rare), which may select an unchanged node other
// than bu_j: that node's columns and records are then fetched on the spot.
// Feasibility is monotone within a window (assumes only add), so a node
// phase 1 found infeasible stays infeasible, and racing reads of columns the
// previous batch's phase 2 is writing (two-batch window) only ever see a
// state between the window start and the live state.

// Workgroup barrier for LDS hand-offs only: wait for this wave's LDS
// operations, then s_barrier.  __syncthreads() also drains every outstanding
// global load (vmcnt(0)), which would expose the latency of the loads this
// kernel keeps in flight across steps (records two pods ahead, the next top
// set); nothing here reads global memory another wave of the workgroup wrote.
// lds_barrier(): ksched_kernels.h

template <int RM>
struct P2Cand {
  int64_t row[2][SlotLayout<RM>::W];   // batch-state columns (slot row layout), per candidate
  uint64_t key[2];                     // phase-1 argmax keys
  int32_t node[2];                     // -1: none
  uint64_t rec[2][3];                  // phase-1 records of pods t, t+1, t+2 (t = the pod it is a candidate for, + 1)
  int32_t img[2][3];
};

struct KeyPair {
  uint64_t k0, k1;
};

struct P2Fold {
  uint64_t k0;      // best contributed key of the wave
  uint32_t cnt;     // feas1 | live << 8 | lost_t << 16 | lost_a << 24 (each <= 64)
  int32_t kidx;     // slot of k0, -1 if not in this wave
};

template <int RM>
struct SlotVal {
  uint64_t key;     // argmax key on live columns, 0 if infeasible
  uint32_t cnt;
  uint64_t live;    // pack_rec(part, rt, ra) if feasible live, else 0
};

// Pod j+1 on one slot row (sw: the row with the version's delta applied).
template <int RM>
__device__ __forceinline__ SlotVal<RM> slot_eval(const CmProf& cm, const ksg_profile& prof, const ksg_pod& p,
                                                 const PodHot<RM>& h, const P1Stats& s1,
                                                 const int64_t (&sw)[SlotLayout<RM>::W], uint64_t x, int32_t img,
                                                 int node) {
  using SL = SlotLayout<RM>;
  SlotVal<RM> r{0, 0, 0};
  if (!(x >> 63)) return r;
  r.cnt = 1;
  const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff;
  const int64_t mt1 = s1.mt, ma1 = s1.ma;
  bool fits = true;
  if (h.fit_on) {
    fits = sw[SL::PODS] + 1 <= sw[SL::ALLOWED];
#pragma unroll
    for (int q = 0; q < RM; q++) fits = fits && (!((h.req_mask >> q) & 1u) || h.req[q] <= sw[2 * q] - sw[2 * q + 1]);
  }
  if (!fits) {
    r.cnt += (rt == mt1 ? 1u << 16 : 0u) + (ra == ma1 ? 1u << 24 : 0u);
    return r;
  }
  int64_t fs = 0, bs = 0;
  if (cm.fast) {
    cm_scores<RM>(cm, h, sw, fs, bs);
  } else {
    NodeCols L;
    slot_row_cols<RM>(sw, L);
    fs = fit_score(prof, p, L);
    bs = ba_score(prof, p, L);
  }
  const int64_t part = img + fs * h.w_fit + bs * h.w_ba;
  const int64_t nt = mt1 != 0 ? 100 - qdiv(100 * rt, mt1, s1.inv_mt) : 100;
  const int64_t na = ma1 != 0 ? qdiv(100 * ra, ma1, s1.inv_ma) : ra;
  r.key = argmax_key(part + nt * h.w_t + na * h.w_a, node);
  r.cnt += 1u << 8;
  r.live = pack_rec(part, rt, ra);
  return r;
}

// Row word k's delta when pod p is assumed (NodeInfo.AddPod on the columns).
template <int RM>
__device__ __forceinline__ int64_t row_delta(const ksg_pod& p, int k, int R) {
  using SL = SlotLayout<RM>;
  if (k < 2 * RM) return ((k & 1) && (k >> 1) < R) ? p.req[k >> 1] : 0;
  if (k == SL::NZC) return p.nz_cpu;
  if (k == SL::NZM) return p.nz_mem;
  if (k == SL::PODS) return 1;
  return 0;
}

template <int RM, int SLOTS>
__global__ __launch_bounds__(2 * SLOTS) void ksg_batch_phase2p(BatchArgs a) {
  using SL = SlotLayout<RM>;
  constexpr int BLOCK = 2 * SLOTS, NW = BLOCK / 64, SW = SL::W;
  static_assert(SLOTS % 64 == 0 && SLOTS <= KSG_BATCH_MAX, "slots in whole waves");
  static_assert(SW <= 32, "a candidate row is fetched by half a wave");
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ P1Stats s_p1[KSG_BATCH_MAX];
  __shared__ int32_t s_clist[SLOTS];
  __shared__ P2Fold s_fold[2][NW];
  __shared__ P2Cand<RM> s_cand[2];
  __shared__ WRed s_w[NW];
  __shared__ ksg_result s_res[KSG_BATCH_MAX];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s = tid % SLOTS;
  const bool cver = tid >= SLOTS;          // wave-uniform
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R, nb = a.nb;
  const int cm_words = (((N + 31) / 32) + 3) & ~3;
  constexpr int POD_WORDS = sizeof(ksg_pod) / 4;
  uint32_t* s_cm[2] = {reinterpret_cast<uint32_t*>(s_dyn), reinterpret_cast<uint32_t*>(s_dyn) + cm_words};
  ksg_pod* s_pods = reinterpret_cast<ksg_pod*>(s_dyn + 2 * cm_words);
  int32_t* s_prog = s_dyn + 2 * cm_words + nb * POD_WORDS;

  const int n_carry = a.carry_n ? *a.carry_n : 0;
  for (int i = tid; i < 2 * cm_words; i += BLOCK) s_dyn[i] = 0;
  for (int i = tid; i < nb * POD_WORDS; i += BLOCK)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + a.b0)[i];
  for (int i = tid; i < a.prog_len; i += BLOCK) s_prog[i] = a.prog[a.prog_lo + i];
  for (int i = tid; i < nb * (int)(sizeof(P1Stats) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(s_p1)[i] = reinterpret_cast<const int32_t*>(a.p1)[i];
  for (int i = tid; i < (int)(sizeof(ksg_profile) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  __syncthreads();
  const CmProf cm = cm_prof(s_prof);
  const bool ipa_filter = ipa_in_filter(s_prof);
  const bool ipa_score = ((s_prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;

  auto rec_at = [&](int j, int n) -> uint64_t { return a.rec[(size_t)j * N + n]; };
  auto img_at = [&](int j, int n) -> int32_t { return a.img[(size_t)j * N + n]; };
  auto clampj = [&](int j) { return j < nb ? j : nb - 1; };
  // word k of node n's slot row (batch-state columns)
  auto row_word = [&](int k, int n) -> int64_t {
    const SlotFetch<RM> f = slot_word_fetch<RM>(c, a.st, k, R, n);
    return slot_word_value<RM>(f, k, R);
  };

  // ---- per-lane slot state -------------------------------------------------
  int nc = n_carry;                 // |C|, block-uniform
  int my_node = 0;
  int64_t row[SW];
#pragma unroll
  for (int k = 0; k < SW; k++) row[k] = 0;
  uint64_t rec1 = 0, rec2 = 0;      // my node's records of pods (t+1, t+2) at step t
  int32_t img1 = 0, img2 = 0;
  uint64_t prv_live = 0;            // my contributed live record of the pod being decided
  bool prv_on = false;
  bool touched = false;             // a pod of this batch was assumed onto my slot
  if (s < n_carry) {
    my_node = a.carry[s];
#pragma unroll
    for (int k = 0; k < SW; k++) row[k] = row_word(k, my_node);
    rec1 = rec_at(0, my_node);
    img1 = img_at(0, my_node);
    rec2 = rec_at(clampj(1), my_node);
    img2 = img_at(clampj(1), my_node);
    if (!cver) {
      s_clist[s] = my_node;
      atomicOr(&s_cm[0][my_node >> 5], 1u << (my_node & 31));
      atomicOr(&s_cm[1][my_node >> 5], 1u << (my_node & 31));
    }
  }
  // top-set keys of the pod whose candidates the next step computes
  uint64_t tk[4];
  auto load_top = [&](int j) {
    const int K = s_p1[j].K;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = lane + 64 * q;
      tk[q] = i < K ? a.top[(size_t)j * KSG_BATCH_MAX + i] : 0;
    }
  };
  // candidates for bu of pod jc: the first two entries of T_jc outside the
  // changed set (cmask); returns their keys (0: none)
  auto candidates = [&](int jc, const uint32_t* cmask) -> KeyPair {
    const int K = s_p1[jc].K;
    uint64_t mk[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = lane + 64 * q;
      bool ok = false;
      if (i < K) {
        const int n = key_node(tk[q]);
        ok = !((cmask[n >> 5] >> (n & 31)) & 1u);
      }
      mk[q] = __ballot(ok);
    }
    int found = 0;
    uint64_t ck[2] = {0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint64_t m = mk[q];
      while (m && found < 2) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        ck[found++] = readlane64(tk[q], l);
      }
    }
    return KeyPair{found > 0 ? ck[0] : 0, found > 1 ? ck[1] : 0};
  };
  // issue the candidate loads (wave 0: rows, half a wave per candidate; the
  // last wave: records), write them into s_cand[buf] after they land
  struct CandLoad {
    int64_t v;
    int kind;   // 0 none, 1 row word, 2 record, 3 img
  };
  // records of pods jc+1, jc+2, jc+3 (the spec lane's pod, then the new
  // slot's next two)
  auto cand_issue = [&](int jc, uint64_t k0, uint64_t k1) -> CandLoad {
    CandLoad L{0, 0};
    const int which = lane >> 5, w = lane & 31;
    const uint64_t kk = which ? k1 : k0;
    if (!kk) return L;
    const int n = key_node(kk);
    if (wv == 0 && w < SW) {
      L.v = row_word(w, n);
      L.kind = 1;
    } else if (wv == NW - 1 && w < 6) {
      const int jj = clampj(jc + 1 + (w % 3));
      if (w < 3) { L.v = (int64_t)rec_at(jj, n); L.kind = 2; }
      else { L.v = img_at(jj, n); L.kind = 3; }
    }
    return L;
  };
  auto cand_store = [&](int buf, uint64_t k0, uint64_t k1, const CandLoad& L) {
    P2Cand<RM>& cb = s_cand[buf];
    const int which = lane >> 5, w = lane & 31;
    if (L.kind == 1) cb.row[which][w] = L.v;
    else if (L.kind == 2) cb.rec[which][w] = (uint64_t)L.v;
    else if (L.kind == 3) cb.img[which][w - 3] = (int32_t)L.v;
    if (tid == 0) {
      cb.key[0] = k0;
      cb.key[1] = k1;
      cb.node[0] = k0 ? key_node(k0) : -1;
      cb.node[1] = k1 ? key_node(k1) : -1;
    }
  };

  // ---- prologue: pod 0 on the carried slots (version N), candidates of pod 0
  {
    load_top(0);
    SlotVal<RM> v{0, 0, 0};
    if (!cver && s < n_carry) {
      const PodHot<RM> h0 = pod_hot<RM>(s_pods[0], s_prof, fit_filter_on, R);
      v = slot_eval<RM>(cm, s_prof, s_pods[0], h0, s_p1[0], row, rec1, img1, my_node);
      prv_on = true;
      prv_live = v.live;
    }
    if (s < n_carry) {   // both versions: the records advance to pods 1, 2
      rec1 = rec2;
      img1 = img2;
      rec2 = rec_at(clampj(2), my_node);
      img2 = img_at(clampj(2), my_node);
    }
    {   // the reductions need every lane of the wave active
      const uint64_t k0 = wreduce(v.key, OpMaxU64{});
      const uint32_t wc = wreduce(v.cnt, OpAdd32{});
      const uint64_t mk = __ballot(k0 != 0 && v.key == k0);
      if (lane == 0) s_fold[0][wv] = P2Fold{k0, wc, mk ? wv * 64 + __builtin_ctzll(mk) : -1};
    }
    __syncthreads();   // s_cm initialised
    const KeyPair ck = candidates(0, s_cm[0]);
    const CandLoad L = cand_issue(0, ck.k0, ck.k1);
    // pod 1's top set for the next candidates
    load_top(clampj(1));
    cand_store(0, ck.k0, ck.k1, L);
    __syncthreads();
  }

  int sel_prev = -1;           // pod j-1's node
  int added_prev = 0;          // pod j-1 created a slot
#ifdef KSG_STAMPS
  unsigned long long st_acc[16] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif
  for (int j = 0; j < nb; j++) {
    KSG_STAMP(0);
    const int buf = j & 1, nbuf = buf ^ 1;
    const ksg_pod& p = s_pods[j];
    const P1Stats s1 = s_p1[j];
    const bool more = j + 1 < nb;
    const int jn = more ? j + 1 : j;
    const ksg_pod& pn = s_pods[jn];
    const P1Stats s1n = s_p1[jn];
    const PodHot<RM> hn = pod_hot<RM>(pn, s_prof, fit_filter_on, R);
    const PodHot<RM> hj = pod_hot<RM>(p, s_prof, fit_filter_on, R);

    // ---- bu_j from the candidates (computed at step j - 1 against C_{j-1}) --
    const P2Cand<RM>& cb = s_cand[buf];
    const int cn0 = cb.node[0], cn1 = cb.node[1];
    const int ci = (cn0 >= 0 && cn0 != sel_prev) ? 0 : 1;
    const int bu = ci == 0 ? cn0 : cn1;            // -1: no unchanged feasible node in T_j
    const uint64_t bu_key = bu >= 0 ? cb.key[ci] : 0;

    KSG_STAMP(1);
    // ---- evaluate pod j+1 (both versions; the spec lane on bu_j + pod j) ----
    const bool spec_lane = cver && s == nc;
    SlotVal<RM> cur{0, 0, 0};
    if (more && (s < nc || (spec_lane && bu >= 0))) {
      int64_t sw[SW];
      uint64_t x = rec1;
      int32_t im = img1;
      int node = my_node;
      if (spec_lane) {
#pragma unroll
        for (int k = 0; k < SW; k++) sw[k] = cb.row[ci][k];
        x = cb.rec[ci][0];
        im = cb.img[ci][0];
        node = bu;
      } else {
#pragma unroll
        for (int k = 0; k < SW; k++) sw[k] = row[k];
      }
      if (cver) {
#pragma unroll
        for (int k = 0; k < SW; k++) sw[k] += row_delta<RM>(p, k, R);
      }
      cur = slot_eval<RM>(cm, s_prof, pn, hn, s1n, sw, x, im, node);
    }

    KSG_STAMP(2);
    // ---- candidates of pod j+1 (T_{j+1} vs C_j), loads land in s_cand[nbuf] --
    KeyPair ckn{0, 0};
    CandLoad L{0, 0};
    if (more) {
      ckn = candidates(jn, s_cm[buf]);
      L = cand_issue(jn, ckn.k0, ckn.k1);
      load_top(clampj(j + 2));
    }

    KSG_STAMP(3);
    // ---- fold pod j's contributions, decide ---------------------------------
    uint64_t k0 = 0;
    int32_t kidx = -1;
    int feas1 = 0, live_n = 0, lost_t = 0, lost_a = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const P2Fold o = s_fold[buf][i];
      if (o.k0 > k0) { k0 = o.k0; kidx = o.kidx; }
      feas1 += o.cnt & 0xff;
      live_n += (o.cnt >> 8) & 0xff;
      lost_t += (o.cnt >> 16) & 0xff;
      lost_a += o.cnt >> 24;
    }
    const int unch = s1.nfeas - feas1;
    int nfeas = unch + live_n;
    const bool renorm = (nfeas >= 2 && (s1.err || (hj.w_t && s1.ht - lost_t <= 0) || (hj.w_a && s1.ha - lost_a <= 0))) ||
                        (unch > 0 && bu < 0);
    int selected = -1, idx = -1;
    uint32_t status = 0;
    if (renorm) {
      // full rescan of pod j's records with the live maxima (the slot lanes
      // that contributed hold pod j's live values)
      const PodView v = make_view(c, s_prof, p, s_prog + (p.blob - a.prog_lo), a.prog);
      const uint32_t* cmj = s_cm[buf];
      auto changed = [&](int n) { return ((cmj[n >> 5] >> (n & 31)) & 1u) != 0; };
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
        if (prv_on) visit(prv_live, my_node);
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
          if (nfeas >= 2) {
            status |= KSG_ST_SCORED;
            if (ge) status |= KSG_ST_SCORE_ERROR;
            else selected = key_node(gb);
          } else if (nfeas == 1) {
            selected = key_node(gb);   // the one feasible node (its key is the only non-zero one)
          }
          if (selected >= 0 && changed(selected)) {
            const uint64_t mk = __ballot(prv_on && my_node == selected);
            if (lane == 0) s_w[wv].cmin = mk ? wv * 64 + __builtin_ctzll(mk) : -1;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < NW; i++) idx = max(idx, s_w[i].cmin);
            idx = idx % SLOTS;
          }
          __syncthreads();
        }
      }
    } else if (nfeas == 1) {
      if (unch == 1) {
        selected = bu;
      } else {
        selected = key_node(k0);
        idx = kidx % SLOTS;
      }
    } else if (nfeas >= 2) {
      status |= KSG_ST_SCORED;
      if (bu_key > k0) {
        selected = bu;
      } else {
        selected = key_node(k0);
        idx = kidx % SLOTS;
      }
    }
    const bool added = selected >= 0 && idx < 0;
    const int slot_j = added ? nc : idx;     // slot pod j lands on (-1: none)
    KSG_STAMP(4);

    // ---- a renormalised choice of an unchanged node other than bu_j: fetch
    // its columns and records now and redo the spec lane (rare) -------------
    if (added && selected != bu) {
      if (s == nc && more) {
        int64_t sw[SW];
#pragma unroll
        for (int k = 0; k < SW; k++) sw[k] = row_word(k, selected);
        if (cver) {
#pragma unroll
          for (int k = 0; k < SW; k++) sw[k] += row_delta<RM>(p, k, R);
          cur = slot_eval<RM>(cm, s_prof, pn, hn, s1n, sw, rec_at(jn, selected), img_at(jn, selected), selected);
        }
      }
    }

    // ---- pod j+1's contributions: one version per slot ---------------------
    const int nc2 = nc + (added ? 1 : 0);
    const bool on = more && (cver ? s == slot_j : (s < nc2 && s != slot_j));
    {
      const uint64_t key = on ? cur.key : 0;
      const uint32_t cnt = on ? cur.cnt : 0;
      const uint64_t kk = wreduce(key, OpMaxU64{});
      const uint32_t wc = wreduce(cnt, OpAdd32{});
      const uint64_t mk = __ballot(kk != 0 && key == kk);
      if (lane == 0) s_fold[nbuf][wv] = P2Fold{kk, wc, mk ? wv * 64 + __builtin_ctzll(mk) : -1};
    }
    prv_on = on;
    prv_live = on ? cur.live : 0;
    KSG_STAMP(5);

    // ---- results, count tables ---------------------------------------------
    if (tid == 0) {
      const bool has_commit = p.commit >= 0;
      if (has_commit && selected >= 0) {   // PodTopologySpread / InterPodAffinity count tables
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
      const bool ipa_none = p.ipa < 0;
      const uint32_t st_pf = ipa_none && ipa_filter ? KSG_ST_IPA_PREFILTER_SKIP : 0u;
      const bool ps_skip = ipa_none && ipa_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u);
      const bool sc = (status & KSG_ST_SCORED) != 0;
      ksg_result res;
      res.selected = selected;
      res.n_feasible = nfeas;
      res.status = status | st_pf | (sc && ps_skip ? KSG_ST_IPA_PRESCORE_SKIP : 0u);
      res.score_skip = p.score_skip | (sc && ps_skip ? bit(KSG_PL_INTER_POD_AFFINITY) : 0u);
      s_res[j] = res;
      // changed set for step j + 1 (the other copy; this step read s_cm[buf])
      if (added_prev) s_cm[nbuf][sel_prev >> 5] |= 1u << (sel_prev & 31);
      if (added) {
        s_cm[nbuf][selected >> 5] |= 1u << (selected & 31);
        s_clist[nc] = selected;
      }
    }

    KSG_STAMP(6);
    // ---- assume pod j on its slot ------------------------------------------
    if (s == slot_j && slot_j >= 0) {
      touched = true;
      if (added) {
        my_node = selected;
        if (selected == bu) {
#pragma unroll
          for (int k = 0; k < SW; k++) row[k] = cb.row[ci][k];
          rec1 = cb.rec[ci][1];
          img1 = cb.img[ci][1];
          rec2 = cb.rec[ci][2];
          img2 = cb.img[ci][2];
        } else {
#pragma unroll
          for (int k = 0; k < SW; k++) row[k] = row_word(k, selected);
          rec1 = rec_at(clampj(j + 2), selected);
          img1 = img_at(clampj(j + 2), selected);
          rec2 = rec_at(clampj(j + 3), selected);
          img2 = img_at(clampj(j + 3), selected);
        }
      } else {
        rec1 = rec2;
        img1 = img2;
        rec2 = rec_at(clampj(j + 3), my_node);
        img2 = img_at(clampj(j + 3), my_node);
      }
#pragma unroll
      for (int k = 0; k < SW; k++) row[k] += row_delta<RM>(p, k, R);
    } else if (s < nc) {
      rec1 = rec2;
      img1 = img2;
      rec2 = rec_at(clampj(j + 3), my_node);
      img2 = img_at(clampj(j + 3), my_node);
    }
    nc = nc2;
    sel_prev = selected;
    added_prev = added ? 1 : 0;
    KSG_STAMP(7);
    if (more) cand_store(nbuf, ckn.k0, ckn.k1, L);
    KSG_STAMP(8);
    lds_barrier();
    KSG_STAMP(9);
  }
#ifdef KSG_STAMPS
  if (tid == 0 && a.stamps)
    for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], st_acc[i]);
#endif

  // ---- write back: the changed nodes' columns, results, the carry list ----
  // (the next batch carries the nodes THIS batch assumed onto: its phase 1
  // read a state at least as new as this batch's start)
  if (!cver && s < nc) {
#pragma unroll
    for (int q = 0; q < RM; q++)
      if (q < R) a.st.requested[(size_t)q * N + my_node] = row[2 * q + 1];
    a.st.nonzero[my_node] = row[SL::NZC];
    a.st.nonzero[(size_t)N + my_node] = row[SL::NZM];
    a.st.pod_count[my_node] = (int32_t)row[SL::PODS];
  }
  if (a.carry_out) {
    const bool t = !cver && s < nc && touched;
    const uint64_t m = __ballot(t);
    if (lane == 0) s_w[wv].cmin = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int i = 0; i < wv; i++) base += s_w[i].cmin;
    if (t) a.carry_out[base + __popcll(m & ((1ull << lane) - 1))] = my_node;
    if (tid == 0) {
      int tot = 0;
      for (int i = 0; i < NW; i++) tot += s_w[i].cmin;
      *a.carry_out_n = tot;
    }
  }
  for (int i = tid; i < nb; i += BLOCK) {
    a.placements[a.out0 + i] = s_res[i].selected;
    if (a.results) a.results[a.out0 + i] = s_res[i];
  }
  for (int i = tid; i < 2 * nb; i += BLOCK) a.pmax[i] = 0;   // ready for this buffer's next phase 1
}
