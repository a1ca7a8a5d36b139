// Phase 2, the one-wave slot walk (KSG_BATCH_MODE "window", the default since
// round 3; included by ksched.hip inside its anonymous namespace, after
// ksg_batch_phase2s).
//
// The slot walk of ksg_batch_phase2s with one lane per changed slot needs
// nb + carried lanes, i.e. two waves at 64-pod batches with the two-batch
// window, and the two waves meet at an LDS barrier every pod: each publishes
// its partial (best changed key, counters) to LDS, waits for the other, and
// both take the same decision.  The stamped build put that exchange (barrier +
// reading the partials + deciding) at a quarter of a pod's cycles
// (profiles/r2/stamps_window_onebarrier.txt).  Here ONE wave walks the batch
// and every lane owns two slots, s = lane and s = lane + 64 (carried + new <=
// 128): the two evaluations are independent, so they interleave in the
// lane's instruction stream instead of running on a second wave, and the
// reductions end in registers (DPP), so a pod needs no barrier and no LDS
// round trip between evaluating and deciding.  Rows and the changed-node
// bitmap stay in LDS, written and read by this wave only (in program order).
//
// Everything else is the slot walk's: phase-1 records and top sets from the
// side stream, the speculated best unchanged node from the sorted top set,
// next-pod loads issued a pod ahead, the exact Fit / BalancedAllocation
// re-evaluation of changed nodes, the renormalisation rescan when a phase-1
// maximum lost every holder, carried slots of the previous batch.  Results
// are the sequential ones bit for bit (tests/test_gpu_batch_variants.py).

template <int RM, bool N32>
__global__ __launch_bounds__(64) void ksg_batch_phase2w(BatchArgs a) {
  using SL = SlotLayout<RM>;
  constexpr int SW = SL::W, SPL = 2, MAXS = 64 * SPL;
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ P1Stats s_p1[64];
  __shared__ int32_t s_clist[MAXS];
  __shared__ ksg_result s_res[64];             // per-pod results, stored after the walk
  __shared__ uint8_t s_touched[MAXS];          // two-batch window: slot assumed onto in this batch

  const int lane = threadIdx.x, tid = lane;
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  const int cm_words = (((N + 31) / 32) + 3) & ~3;
  constexpr int POD_WORDS = sizeof(ksg_pod) / 4;
  uint32_t* s_cmask = reinterpret_cast<uint32_t*>(s_dyn);
  ksg_pod* s_pods = reinterpret_cast<ksg_pod*>(s_dyn + cm_words);
  int32_t* s_prog = s_dyn + cm_words + a.nb * POD_WORDS;
  int64_t* s_slot = reinterpret_cast<int64_t*>(s_dyn + ((cm_words + a.nb * POD_WORDS + a.prog_len + 3) & ~3));

  for (int i = tid; i < cm_words; i += 64) s_cmask[i] = 0;
  for (int i = tid; i < a.nb * POD_WORDS; i += 64)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + a.b0)[i];
  for (int i = tid; i < a.prog_len; i += 64) s_prog[i] = a.prog[a.prog_lo + i];
  for (int i = tid; i < a.nb * (int)(sizeof(P1Stats) / 4); i += 64)
    reinterpret_cast<int32_t*>(s_p1)[i] = reinterpret_cast<const int32_t*>(a.p1)[i];
  for (int i = tid; i < (int)(sizeof(ksg_profile) / 4); i += 64)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  __syncthreads();
  const CmProf cm = cm_prof(s_prof);
  const bool ipa_filter = ipa_in_filter(s_prof);
  const bool ipa_score = ((s_prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;
  const SlotPlan plan = slot_plan<RM, N32>(c, a.st, lane, R);

  auto changed = [&](int n) { return ((s_cmask[n >> 5] >> (n & 31)) & 1u) != 0; };
  int nc = 0;                          // |C|, wave-uniform
  int my_node[SPL] = {0, 0};           // node of slot lane + 64 q (slot < nc)
  uint64_t my_rec[SPL] = {0, 0};       // pod j's phase-1 record at my_node[q]
  int32_t my_img[SPL] = {0, 0};
  int32_t my_stat[SPL] = {0, 0};       // N32: pod j's static part of the total (a.stat)
  if (a.carry) {   // the previous batch's nodes start as slots with their live rows
    nc = *a.carry_n;
    for (int t = tid; t < nc * SW; t += 64) {
      const int i = t / SW, w = t - i * SW;
      const SlotFetch<RM> f = slot_word_fetch<RM, N32>(c, a.st, w, R, a.carry[i]);
      s_slot[(size_t)i * SL::STRIDE + w] = slot_word_value<RM, N32>(f, w, R);
    }
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const int s = lane + 64 * q;
      if (s < nc) {
        my_node[q] = a.carry[s];
        s_clist[s] = my_node[q];
        atomicOr(&s_cmask[my_node[q] >> 5], 1u << (my_node[q] & 31));
        my_rec[q] = a.rec[my_node[q]];
        my_img[q] = a.img[my_node[q]];
        if constexpr (N32) my_stat[q] = a.stat[my_node[q]];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < SPL; q++) s_touched[lane + 64 * q] = 0;
  __syncthreads();
  uint64_t t64 = a.top[lane];
  bool t_chg = lane < s_p1[0].K ? changed(key_node(t64)) : true;
  int prev_sel = -1;
  for (int j = 0; j < a.nb; j++) {
    const ksg_pod& p = s_pods[j];
    const ksg_profile& prof = s_prof;
    const P1Stats s1 = s_p1[j];
    const PodHot<RM> h = pod_hot<RM>(p, prof, fit_filter_on, R);
    const int rl = (lane >> 1) < RM ? (lane >> 1) : 0;
    const int64_t req_l = p.req[rl];
    const int32_t p_commit = p.commit, p_ipa = p.ipa;
    const uint32_t p_skip = p.score_skip;
    const int64_t row_delta = lane < 2 * RM ? ((lane & 1) && (lane >> 1) < R ? req_l : 0)
                              : lane == SL::NZC ? h.nz_cpu
                              : lane == SL::NZM ? h.nz_mem
                              : lane == SL::PODS ? 1 : 0;
    const bool has_commit = p_commit >= 0;
    const bool ipa_none = p_ipa < 0;
    const uint32_t st_pf = ipa_none && ipa_filter ? KSG_ST_IPA_PREFILTER_SKIP : 0u;
    const bool ps_skip = ipa_none && ipa_score && !((p_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u);
    const uint32_t pod_status = st_pf, pod_skip = p_skip;
    const uint32_t pod_status_s = KSG_ST_SCORED | st_pf | (ps_skip ? KSG_ST_IPA_PRESCORE_SKIP : 0u);
    const uint32_t pod_skip_s = p_skip | (ps_skip ? bit(KSG_PL_INTER_POD_AFFINITY) : 0u);
    const int64_t mt1 = s1.mt, ma1 = s1.ma;
    const bool more = j + 1 < a.nb;
    const int jn = more ? j + 1 : j;

    // ---- X1: speculated best unchanged node (sorted T_j, first 64 entries) --
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
    // ---- X2: pod j+1's loads (consumed at the assume) ----------------------
    const int K1 = more ? s_p1[j + 1].K : 0;
    uint64_t nx_rec[SPL];
    int32_t nx_img[SPL], nx_stat[SPL];
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const int s = lane + 64 * q;
      const int nn = s < nc ? my_node[q] : (spec >= 0 ? spec : 0);
      nx_rec[q] = a.rec[(size_t)jn * N + nn];
      nx_img[q] = a.img[(size_t)jn * N + nn];
      nx_stat[q] = 0;
      if constexpr (N32) nx_stat[q] = a.stat[(size_t)jn * N + nn];
    }
    const uint64_t nx_t64 = a.top[(size_t)jn * KSG_BATCH_MAX + lane];
    SlotFetch<RM> col = slot_plan_fetch<RM>(plan, spec >= 0 ? spec : 0);

    // ---- X3: my changed nodes on their live rows -------------------------------
    uint32_t cnt = 0;   // feas1 | live << 8 | lost_t << 16 | lost_a << 24 (each <= 128)
    uint64_t live[SPL] = {0, 0}, key[SPL] = {0, 0};
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const int s = lane + 64 * q;
      if (!(s < nc && (my_rec[q] >> 63))) continue;
      int64_t sw[SW];
      {
        const int4* src = reinterpret_cast<const int4*>(s_slot + (size_t)s * SL::STRIDE);
#pragma unroll
        for (int k = 0; k < SW / 2; k++) reinterpret_cast<int4*>(sw)[k] = src[k];
      }
      const uint64_t x = my_rec[q];
      cnt += 1;
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
        int64_t part, total;
        if constexpr (N32) {
          const int32_t fb = (int32_t)fs * (int32_t)h.w_fit + (int32_t)bs * (int32_t)h.w_ba;
          part = my_img[q] + fb;
          total = my_stat[q] + fb;
        } else {
          const int32_t nt = mt1 != 0 ? 100 - qdiv32(100 * (int32_t)rt, (int32_t)mt1, s1.inv_mt) : 100;
          const int32_t na = ma1 != 0 ? qdiv32(100 * (int32_t)ra, (int32_t)ma1, s1.inv_ma) : (int32_t)ra;
          part = my_img[q] + fs * h.w_fit + bs * h.w_ba;
          total = part + nt * h.w_t + na * h.w_a;
        }
        key[q] = argmax_key(total, my_node[q]);
        cnt += 1u << 8;
        live[q] = pack_rec(part, rt, ra);
      }
    }
    // the wave's best changed key and its slot, the counters: registers only
    const uint64_t my_key = key[0] > key[1] ? key[0] : key[1];
    const int my_kslot = key[0] > key[1] ? lane : lane + 64;
    const uint64_t k0 = wreduce(my_key, OpMaxU64{});
    const uint32_t wc = wreduce(cnt, OpAdd32{});
    int32_t kidx = -1;
    {
      const uint64_t mk = __ballot(k0 != 0 && my_key == k0);
      if (mk) kidx = __builtin_amdgcn_readlane(my_kslot, __builtin_ctzll(mk));
    }
    uint64_t bu = bu_key;
    if (bu_full) {   // best unchanged of T_j beyond its first 64 entries (rare)
      uint64_t tk = 0;
      for (int e = lane; e < s1.K; e += 64) {
        const uint64_t k = a.top[(size_t)j * KSG_BATCH_MAX + e];
        const int kn = key_node(k);
        if (!changed(kn) && kn != prev_sel && k > tk) tk = k;
      }
      bu = wreduce(tk, OpMaxU64{});
    }

    // ---- Y: decide ---------------------------------------------------------------
    const int feas1 = wc & 0xff, live_n = (wc >> 8) & 0xff, lost_t = (wc >> 16) & 0xff, lost_a = wc >> 24;
    const int unch = s1.nfeas - feas1;   // unchanged feasible nodes
    int nfeas = unch + live_n;
    const bool renorm = nfeas >= 2 && (s1.err || (h.w_t && s1.ht - lost_t <= 0) || (h.w_a && s1.ha - lost_a <= 0));
    int selected = -1, idx = -1;   // idx: slot of the selected node if it is in C
    uint32_t status = 0;
    if (renorm) {   // renormalise with the live maxima over all of pod j's records (rare)
      const PodView v = make_view(c, prof, p, s_prog + (p.blob - a.prog_lo), a.prog);
      const uint64_t* rec = a.rec + (size_t)j * N;
      int64_t gmt = 0, gma = 0;
      int32_t gn = 0;
      for (int pass = 0; pass < 2; pass++) {
        uint64_t best = 0;
        uint32_t err = 0;
        int64_t lmt = 0, lma = 0;
        int32_t ln = 0;
        auto visit = [&](uint64_t x, int n) {
          if (!(x >> 63)) return;
          const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
          if (pass == 0) {
            ln += 1;
            lmt = max(lmt, rt);
            lma = max(lma, ra);
          } else {
            const uint64_t k = argmax_key(total_score(v, part, rt, ra, gmt, gma, err, nullptr, nullptr), n);
            best = k > best ? k : best;
          }
        };
        for (int n = lane; n < N; n += 64)
          if (!changed(n)) visit(rec[n], n);
#pragma unroll
        for (int q = 0; q < SPL; q++)
          if (lane + 64 * q < nc) visit(live[q], my_node[q]);
        if (pass == 0) {
          gmt = wreduce(lmt, OpMax64{});
          gma = wreduce(lma, OpMax64{});
          gn = (int32_t)wreduce((uint32_t)ln, OpAdd32{});
        } else {
          const uint64_t gb = wreduce(best, OpMaxU64{});
          const uint32_t ge = wreduce(err, OpOr32{});
          nfeas = gn;
          status |= KSG_ST_SCORED;
          if (ge) status |= KSG_ST_SCORE_ERROR;
          else selected = key_node(gb);
          if (selected >= 0 && changed(selected)) {
            int mys = -1;
#pragma unroll
            for (int q = 0; q < SPL; q++)
              if (lane + 64 * q < nc && my_node[q] == selected) mys = lane + 64 * q;
            const uint64_t mk = __ballot(mys >= 0);
            idx = __builtin_amdgcn_readlane(mys, __builtin_ctzll(mk));
          }
        }
      }
    } else if (nfeas == 1) {
      if (unch == 1) {
        selected = key_node(bu);
      } else {   // the one live changed node (rare)
        int mys = -1;
#pragma unroll
        for (int q = 0; q < SPL; q++)
          if (lane + 64 * q < nc && live[q] != 0) mys = lane + 64 * q;
        const uint64_t mb = __ballot(mys >= 0);
        idx = __builtin_amdgcn_readlane(mys, __builtin_ctzll(mb));
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

    // ---- Y: assume -------------------------------------------------------------
    const bool added = selected >= 0 && idx < 0;
    const int nq = nc >> 6, nl = nc & 63;   // the new slot's half and lane
    if (added && selected != spec) {        // speculation missed: dependent loads
      col = slot_plan_fetch<RM>(plan, selected);
      if (lane == nl) {
#pragma unroll
        for (int q = 0; q < SPL; q++)
          if (q == nq) {
            nx_rec[q] = a.rec[(size_t)jn * N + selected];
            nx_img[q] = a.img[(size_t)jn * N + selected];
            if constexpr (N32) nx_stat[q] = a.stat[(size_t)jn * N + selected];
          }
      }
    }
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const int s = lane + 64 * q;
      if (added && s == nc) my_node[q] = selected;
      if (s < nc + (added ? 1 : 0)) {
        my_rec[q] = nx_rec[q];
        my_img[q] = nx_img[q];
        my_stat[q] = nx_stat[q];
      }
    }
    t64 = nx_t64;
    t_chg = lane < K1 ? (changed(key_node(t64)) || key_node(t64) == selected) : true;
    const int64_t col_val = slot_word_value<RM, N32>(col, lane, R);
    const int slot = added ? nc : idx;
    if (selected >= 0) {
      int64_t* row = s_slot + (size_t)slot * SL::STRIDE;
      if (added) {
        if (lane < SW) row[lane] = col_val + row_delta;
      } else if (lane < SW && row_delta != 0) {   // an LDS add without return: nothing waits on it
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
    if (lane == 0) {
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
  }
  __syncthreads();
  for (int i = tid; i < nc * SW; i += 64) {
    const int slot = i / SW, w = i - slot * SW, node = s_clist[slot];
    const int64_t val = s_slot[(size_t)slot * SL::STRIDE + w];
    if (w < 2 * RM && (w & 1) && (w >> 1) < R) a.st.requested[(size_t)(w >> 1) * N + node] = val;
    else if (w == SL::NZC || w == SL::NZM) a.st.nonzero[(size_t)(w - SL::NZC) * N + node] = val;
    else if (w == SL::PODS) a.st.pod_count[node] = (int32_t)val;
  }
  for (int i = tid; i < a.nb; i += 64) {
    a.placements[a.out0 + i] = s_res[i].selected;
    if (a.results) a.results[a.out0 + i] = s_res[i];
  }
  for (int i = tid; i < 2 * a.nb; i += 64) a.pmax[i] = 0;   // ready for the next batch's phase 1
  if (a.carry_out) {   // the nodes this batch touched, in slot order, for the next batch
    int base = 0;
#pragma unroll
    for (int q = 0; q < SPL; q++) {
      const int s = lane + 64 * q;
      const bool t = s < nc && s_touched[s];
      const uint64_t m = __ballot(t);
      if (t) a.carry_out[base + __popcll(m & ((1ull << lane) - 1))] = s_clist[s];
      base += (int)__popcll(m);
    }
    if (lane == 0) *a.carry_out_n = base;
  }
}
