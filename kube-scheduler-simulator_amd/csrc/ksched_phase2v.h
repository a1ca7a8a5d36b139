// Phase 2, speculate-and-verify walk (KSG_BATCH_MODE=spec), included by
// ksched.hip after ksched_phase2t.h (it reuses the transposed walk's N32
// column evaluation: TcPod / TcRow / tc_eval).
//
// The slot walk and the transposed walk both put one exact evaluation of a
// changed node on every pod's critical path.  On configs[1] about 97 % of the
// pods take their best UNCHANGED node (the first entry of the top set T_j
// outside the changed set D_j), which needs no evaluation at all: it follows
// from the top sets and from which nodes earlier pods took.  So each round:
//
//   1. speculate (wave 0, lane q = pod q): from `start` on, every pod takes its
//      best unchanged node.  Lane q keeps a pointer into T_q (staged in LDS)
//      past every entry already in D; per pod k one v_readlane gives d_k, the
//      lanes whose candidate is d_k step their pointer on (LDS reads of T and
//      of the changed bitmap).  No evaluation on this chain.  Every lane's
//      pointer is snapshotted per step (a rollback restores it).
//   2. versions (all waves): pod k's assume onto d_k creates a new slot with
//      one row version, node d_k's live columns + pod k's deltas (one global
//      fetch per word, one thread per (pod, word)).
//   3. verify (all waves, lane = pod): every row version v of every changed
//      slot (carried slots' live rows, earlier rounds' committed versions,
//      this round's speculated ones) is visible to the pods in (t_v, t_next];
//      each wave evaluates its versions for all 64 pods at once (the N32
//      Fit / BalancedAllocation of tc_eval, phase-1 records from the
//      node-major copies) and folds them into per-pod LDS maxima and counters
//      (ds_max_u64 / ds_add_u32).
//   4. check (wave 0): each pod's exact decision from its counters, best column
//      and best unchanged key, exactly as the slot walk decides it.  The first
//      pod k* whose decision differs from the speculated one (or that needs the
//      renormalisation rescan) ends the round: pods before it are committed,
//      k*'s exact decision is applied (a new version of an existing slot, or a
//      new slot), the speculated slots after it are dropped, and the next
//      round speculates from k* + 1 with the pointers restored from k*'s
//      snapshot.
//
// Every decision equals the sequential one: a pod's decision is committed only
// after verification against the state every earlier committed decision left,
// and k*'s decision is computed from that same verified state.  Results equal
// the slot walk's and the oracle's bit for bit.
//
// Scope (host: run_pipe, mode 6): the transposed walk's (N32 ranges, compact
// Fit / BalancedAllocation profile, <= 64-pod batches in the two-batch window).

constexpr int kSvWaves = 16;                  // 1024 lanes
constexpr int kSvSlots = 2 * 64;              // carried (<= previous batch) + this batch's
constexpr int kSvRow = SlotLayout<4>::STRIDE; // int64 words per LDS row

__device__ __forceinline__ bool sv_changed(const uint32_t* cm, int n) { return ((cm[n >> 5] >> (n & 31)) & 1u) != 0; }

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ksg_batch_phase2v(BatchArgs a) {
  using SL = SlotLayout<4>;
  constexpr int NW = BLOCK / 64;
  constexpr int SW = SL::W;
  static_assert(BLOCK == 64 * kSvWaves && SW == 16 && 64 * SW == BLOCK, "one thread per (pod, row word)");
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ __attribute__((aligned(16))) TcU s_u[64];
  __shared__ ksg_result s_res[64];
  __shared__ int32_t s_clist[kSvSlots];   // node of slot (-1: a hole, pod without a node)
  __shared__ int32_t s_lastv[kSvSlots];   // newest version of slot
  __shared__ int32_t s_vslot[kSvSlots];   // slot of version (-1: hole)
  __shared__ int32_t s_vt[kSvSlots];      // pod whose assume made the version (-1: carried live row)
  __shared__ int32_t s_vnext[kSvSlots];   // next version of the same slot, -1 if newest
  __shared__ int32_t s_dec[64];           // pod's node (speculated, then committed)
  __shared__ int32_t s_dslot[64];         // slot of s_dec, -1 if none
  __shared__ uint64_t s_bu[64];           // pod's best unchanged key (0: none)
  __shared__ uint64_t s_best[64];         // verification: best live column key
  __shared__ uint32_t s_cnt[64];          // verification: p1 feasible | live << 8 | lost taint << 16 | lost aff << 24
  __shared__ uint8_t s_snap[64 * 64];     // [step][pod] T pointer before the step's conflicts
  __shared__ int32_t s_ctl[4];            // round control: next start, k*

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const DevCluster& c = a.c;
  const int N = c.N, R = c.R;
  const int nb = a.nb;
  const int cm_words = (((N + 31) / 32) + 3) & ~3;
  constexpr int POD_WORDS = sizeof(ksg_pod) / 4;
  const int KT = nb + a.k_extra;   // T stride in LDS (entries): K = min(j + 1 + k_extra, nfeas)
  uint32_t* s_cmask = reinterpret_cast<uint32_t*>(s_dyn);
  ksg_pod* s_pods = reinterpret_cast<ksg_pod*>(s_dyn + cm_words);
  int32_t* s_prog = s_dyn + cm_words + nb * POD_WORDS;
  int64_t* s_vrow = reinterpret_cast<int64_t*>(s_dyn + ((cm_words + nb * POD_WORDS + a.prog_len + 3) & ~3));
  int32_t* s_top = reinterpret_cast<int32_t*>(s_vrow + (size_t)kSvSlots * kSvRow);   // [64][KT] nodes

  if (a.tk_done) {   // this batch's phase 1 / top-k / transpose (second stream) are done: poll, then acquire
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
  for (int i = tid; i < nb * POD_WORDS; i += BLOCK)
    reinterpret_cast<int32_t*>(s_pods)[i] = reinterpret_cast<const int32_t*>(a.pods + a.b0)[i];
  for (int i = tid; i < a.prog_len; i += BLOCK) s_prog[i] = a.prog[a.prog_lo + i];
  for (int i = tid; i < (int)(sizeof(ksg_profile) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  // T as node indices, [pod][KT]
  for (int x = tid; x < nb * KT; x += BLOCK) {
    const int q = x / KT, i = x - q * KT;
    const int K = a.p1[q].K;
    s_top[x] = i < K ? key_node(a.top[(size_t)q * KSG_BATCH_MAX + i]) : -1;
  }
  const int nc0 = a.carry ? *a.carry_n : 0;
  // carried slots: version t = slot t = the live row of carried node t
  for (int x = tid; x < nc0 * SW; x += BLOCK) {
    const int t = x / SW, w = x - t * SW;
    const int d = a.carry[t];
    s_vrow[(size_t)t * kSvRow + w] = slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, w, R, d), w, R);
    if (w == 0) {
      s_clist[t] = d;
      s_lastv[t] = t;
      s_vslot[t] = t;
      s_vt[t] = -1;
      s_vnext[t] = -1;
    }
  }
  __syncthreads();
  const ksg_profile& prof = s_prof;
  const TcProf cm = tc_prof(cm_prof(prof));
  const bool ipa_filter = ipa_in_filter(prof);
  const bool ipa_score = ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;
  for (int t = tid; t < nc0; t += BLOCK) atomicOr(&s_cmask[a.carry[t] >> 5], 1u << (a.carry[t] & 31));
  // lane q's pod (every wave: the verification evaluates for every pod)
  const int qq = lane < nb ? lane : 0;
  const TcPod hp = tc_pod(s_pods[qq], prof, a.p1[qq], fit_filter_on, R);
  if (wv == 0 && lane < nb) {
    const ksg_pod& p = s_pods[lane];
    const P1Stats s1 = a.p1[lane];
    const uint32_t smask = prof.score_mask & ~p.score_skip;
    TcU u;
#pragma unroll
    for (int r = 0; r < 4; r++) u.req[r] = r < R ? p.req[r] : 0;
    u.nzc = p.nz_cpu;
    u.nzm = p.nz_mem;
    u.nfeas = s1.nfeas;
    u.K = s1.K;
    u.ht = s1.ht;
    u.ha = s1.ha;
    const bool wt = (smask & bit(KSG_PL_TAINT_TOLERATION)) && prof.weight[KSG_PL_TAINT_TOLERATION];
    const bool wa = (smask & bit(KSG_PL_NODE_AFFINITY)) && prof.weight[KSG_PL_NODE_AFFINITY];
    u.flags = (s1.err ? 1u : 0u) | (wt ? 2u : 0u) | (wa ? 4u : 0u) | (p.commit >= 0 ? 8u : 0u);
    const bool ipa_none = p.ipa < 0;
    const bool ps_skip = ipa_none && ipa_score && !((p.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u);
    u.st_pf = ipa_none && ipa_filter ? KSG_ST_IPA_PREFILTER_SKIP : 0u;
    u.st_sc = KSG_ST_SCORED | (ps_skip ? KSG_ST_IPA_PRESCORE_SKIP : 0u);
    u.skip = p.score_skip;
    u.skip_sc = p.score_skip | (ps_skip ? bit(KSG_PL_INTER_POD_AFFINITY) : 0u);
    u.pad[0] = u.pad[1] = u.pad[2] = 0;
    s_u[lane] = u;
  }
  __syncthreads();
  // initial pointers: T_q's first entry outside the carried nodes (wave w: pods w, w + NW, ...)
  for (int q = wv; q < nb; q += NW) {
    const int K = a.p1[q].K;
    int ptr = K;
    for (int b = 0; b < K && ptr == K; b += 64) {
      const int i = b + lane;
      const int n = i < K ? s_top[q * KT + i] : -1;
      const uint64_t m = __ballot(i < K && !sv_changed(s_cmask, n));
      if (m) ptr = b + __builtin_ctzll(m);
    }
    if (lane == 0) s_snap[q] = (uint8_t)ptr;   // step 0's row of the snapshot = the round-1 pointers
  }
  __syncthreads();

  // This lane's pod's row delta word `w` (the assume: requested += req, nonzero, pod count)
  auto delta_word = [&](const TcU& u, int w) -> int64_t {
    const int rl = (w >> 1) & 3;
    const int64_t req_l = rl == 0 ? u.req[0] : rl == 1 ? u.req[1] : rl == 2 ? u.req[2] : u.req[3];
    return w < 8 ? ((w & 1) ? req_l : 0) : w == SL::NZC ? u.nzc : w == SL::NZM ? u.nzm : w == SL::PODS ? 1 : 0;
  };

  int start = 0;
  int nv_c = nc0, ns_c = nc0;   // committed versions / slots (uniform)
  // wave 0's speculation state: lane q's pointer into T_q and its node (-1: none)
  int ptr = 0, cnode = -1;
  if (wv == 0 && lane < nb) {
    ptr = s_snap[lane];
    cnode = ptr < s_u[lane].K ? s_top[lane * KT + ptr] : -1;
  }
  int guard = 0;
  while (start < nb && guard++ <= nb) {
    // ---- 1. speculate (wave 0) ---------------------------------------------------
    if (wv == 0) {
      const int Kq = lane < nb ? s_u[lane].K : 0;
      for (int k = start; k < nb; k++) {
        s_snap[k * 64 + lane] = (uint8_t)ptr;
        const int d = __builtin_amdgcn_readlane(cnode, k);
        if (d < 0) continue;
        if (lane == 0) s_cmask[d >> 5] |= 1u << (d & 31);
        bool conflict = lane > k && lane < nb && cnode == d;
        while (__ballot(conflict)) {
          if (conflict) {
            ptr++;
            cnode = ptr < Kq ? s_top[lane * KT + ptr] : -1;
            conflict = cnode >= 0 && sv_changed(s_cmask, cnode);
          }
        }
      }
    }
    __syncthreads();
    // ---- 2. this round's versions: thread (pod k, word w) ------------------------
    {
      const int k = tid >> 4, w = tid & 15;
      if (k >= start && k < nb) {
        const int pk = s_snap[k * 64 + k];
        const int d = pk < s_u[k].K ? s_top[k * KT + pk] : -1;
        const int v = nv_c + (k - start), s = ns_c + (k - start);
        if (d >= 0) {
          const int64_t base = slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, w, R, d), w, R);
          s_vrow[(size_t)v * kSvRow + w] = base + delta_word(s_u[k], w);
        }
        if (w == 0) {
          s_dec[k] = d;
          s_dslot[k] = d >= 0 ? s : -1;
          s_bu[k] = d >= 0 ? a.top[(size_t)k * KSG_BATCH_MAX + pk] : 0;
          s_clist[s] = d;
          s_lastv[s] = v;
          s_vslot[v] = d >= 0 ? s : -1;
          s_vt[v] = k;
          s_vnext[v] = -1;
          s_best[k] = 0;
          s_cnt[k] = 0;
        }
      }
    }
    __syncthreads();
    const int nv = nv_c + (nb - start);
    // ---- 3. verify: wave w evaluates versions w, w + NW, ... for every pod --------
    {
      const bool mine = lane < nb && lane >= start;
      for (int v = wv; v < nv; v += NW) {
        const int s = s_vslot[v];
        if (s < 0) continue;
        const int t_lo = s_vt[v], vn = s_vnext[v];
        const int t_hi = vn >= 0 ? s_vt[vn] : nb - 1;
        if (t_hi < start) continue;
        const int node = s_clist[s];
        const uint64_t x = a.rect[(size_t)node * 64 + lane];
        const int32_t stat = a.statt[(size_t)node * 64 + lane];
        int64_t w[SW];
        {
          const int4* src = reinterpret_cast<const int4*>(s_vrow + (size_t)v * kSvRow);
#pragma unroll
          for (int i = 0; i < SW / 2; i++) reinterpret_cast<int4*>(w)[i] = src[i];
        }
        const TcRow row = tc_row(cm, w);
        const bool act = mine && lane > t_lo && lane <= t_hi;
        const bool p1f = (x >> 63) != 0;
        const bool ft = p1f && (int32_t)((x >> 48) & 0xff) == hp.mt;
        const bool fa = p1f && (int32_t)((x >> 32) & 0xffff) == hp.ma;
        int32_t fb = 0;
        const bool live = tc_eval(cm, hp, row, fb) && p1f;
        const uint32_t dc = (p1f ? 1u : 0u) + (live ? 1u << 8 : 0u) + (p1f && !live && ft ? 1u << 16 : 0u) +
                            (p1f && !live && fa ? 1u << 24 : 0u);
        if (act && dc) atomicAdd(&s_cnt[lane], dc);
        if (act && live) atomicMax(reinterpret_cast<unsigned long long*>(&s_best[lane]),
                                   (unsigned long long)argmax_key(stat + fb, node));
      }
    }
    __syncthreads();
    // ---- 4. check + commit (wave 0) ------------------------------------------------
    if (wv == 0) {
      const bool mine = lane < nb && lane >= start;
      const TcU u = s_u[lane < nb ? lane : 0];
      const uint32_t kc = s_cnt[lane];
      const uint64_t k0 = s_best[lane], bu = s_bu[lane];
      const int feas1 = kc & 0xff, live_n = (kc >> 8) & 0xff, lost_t = (kc >> 16) & 0xff, lost_a = kc >> 24;
      const int unch = u.nfeas - feas1;
      const int nfeas = unch + live_n;
      const bool renorm = nfeas >= 2 && ((u.flags & 1u) || ((u.flags & 2u) && u.ht - lost_t <= 0) ||
                                         ((u.flags & 4u) && u.ha - lost_a <= 0));
      int exact = -1;
      if (nfeas == 1) exact = unch == 1 ? key_node(bu) : key_node(k0);
      else if (nfeas >= 2) exact = bu > k0 ? key_node(bu) : key_node(k0);
      const int spec = s_dec[lane < nb ? lane : 0];
      const uint64_t bad = __ballot(mine && (renorm || exact != spec));
      const int ks = bad ? __builtin_ctzll(bad) : nb;
      if (mine && lane < ks) {   // committed as speculated
        const bool sc = nfeas >= 2;
        ksg_result res;
        res.selected = spec;
        res.n_feasible = nfeas;
        res.status = (sc ? KSG_ST_SCORED : 0u) | u.st_pf | (sc ? u.st_sc : 0u);
        res.score_skip = sc ? u.skip_sc : u.skip;
        s_res[lane] = res;
      }
      // the speculated slots of pods k* .. nb - 1 are dropped
      if (mine && lane >= ks && spec >= 0) atomicAnd(&s_cmask[spec >> 5], ~(1u << (spec & 31)));
      nv_c += ks - start;
      ns_c += ks - start;
      if (ks < nb) {
        const int k = ks;
        const TcU uk = s_u[k];
        const bool renorm_k = __builtin_amdgcn_readlane((int)renorm, k) != 0;
        int nfeas_k = __builtin_amdgcn_readlane(nfeas, k);
        int selected = -1;
        uint32_t status = 0;
        if (renorm_k) {   // the renormalisation rescan: pod k over its phase-1 records and the live columns
          const ksg_pod& p = s_pods[k];
          const PodView pv = make_view(c, prof, p, s_prog + (p.blob - a.prog_lo), a.prog);
          const TcPod hk = tc_pod(p, prof, a.p1[k], fit_filter_on, R);
          const uint64_t* rec = a.rec + (size_t)k * N;
          const int32_t* img = a.img + (size_t)k * N;
          auto live_rec = [&](int s) -> uint64_t {   // pod k on slot s's newest committed version
            const int nd = s_clist[s];
            if (nd < 0) return 0;
            const uint64_t x = rec[nd];
            if (!(x >> 63)) return 0;
            int64_t w[SW];
            const int64_t* src = s_vrow + (size_t)s_lastv[s] * kSvRow;
#pragma unroll
            for (int i = 0; i < SW; i++) w[i] = src[i];
            int32_t fb = 0;
            if (!tc_eval(cm, hk, tc_row(cm, w), fb)) return 0;
            return pack_rec((int64_t)img[nd] + fb, (x >> 48) & 0xff, (x >> 32) & 0xffff);
          };
          Red r{0, 0, 0, 0x7fffffff};
          auto fold = [&](uint64_t x) {
            if (!(x >> 63)) return;
            r.nfeas += 1;
            r.max_t = max(r.max_t, (int64_t)((x >> 48) & 0xff));
            r.max_a = max(r.max_a, (int64_t)((x >> 32) & 0xffff));
          };
          for (int n = lane; n < N; n += 64)
            if (!sv_changed(s_cmask, n)) fold(rec[n]);
          for (int s = lane; s < ns_c; s += 64) fold(live_rec(s));
          const int64_t max_t = wreduce(r.max_t, OpMax64{}), max_a = wreduce(r.max_a, OpMax64{});
          nfeas_k = (int)wreduce((uint32_t)r.nfeas, OpAdd32{});
          uint64_t best = 0;
          uint32_t err = 0;
          auto visit = [&](uint64_t x, int n) {
            const int64_t rt = (x >> 48) & 0xff, ra = (x >> 32) & 0xffff, part = (uint32_t)x;
            const uint64_t key = argmax_key(total_score(pv, part, rt, ra, max_t, max_a, err, nullptr, nullptr), n);
            best = key > best ? key : best;
          };
          for (int n = lane; n < N; n += 64) {
            if (sv_changed(s_cmask, n)) continue;
            const uint64_t x = rec[n];
            if (x >> 63) visit(x, n);
          }
          for (int s = lane; s < ns_c; s += 64) {
            const uint64_t x = live_rec(s);
            if (x >> 63) visit(x, s_clist[s]);
          }
          best = wreduce(best, OpMaxU64{});
          err = wreduce(err, OpOr32{});
          status = KSG_ST_SCORED;
          if (err) status |= KSG_ST_SCORE_ERROR;
          else selected = key_node(best);
        } else {
          selected = __builtin_amdgcn_readlane(exact, k);
          status = nfeas_k >= 2 ? KSG_ST_SCORED : 0u;
        }
        // slot of `selected` among the committed slots, -1 if it is a new node
        int idx = -1;
        if (selected >= 0)
          for (int b = 0; b < ns_c && idx < 0; b += 64) {
            const uint64_t mk = __ballot(b + lane < ns_c && s_clist[b + lane] == selected);
            if (mk) idx = b + __builtin_ctzll(mk);
          }
        const int v = nv_c;
        if (selected >= 0) {
          const int s = idx >= 0 ? idx : ns_c;
          if (lane < SW) {
            const int64_t base = idx >= 0 ? s_vrow[(size_t)s_lastv[idx] * kSvRow + lane]
                                          : slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, lane, R, selected),
                                                                     lane, R);
            s_vrow[(size_t)v * kSvRow + lane] = base + delta_word(uk, lane);
          }
          if (lane == 0) {
            if (idx >= 0) s_vnext[s_lastv[idx]] = v;
            else {
              s_clist[s] = selected;
              s_cmask[selected >> 5] |= 1u << (selected & 31);
            }
            s_lastv[s] = v;
            s_vslot[v] = s;
            s_vt[v] = k;
            s_vnext[v] = -1;
            s_dec[k] = selected;
            s_dslot[k] = s;
          }
          nv_c += 1;
          if (idx < 0) ns_c += 1;
        } else if (lane == 0) {
          s_dec[k] = -1;
          s_dslot[k] = -1;
        }
        if (lane == 0) {
          const bool sc = (status & KSG_ST_SCORED) != 0;
          ksg_result res;
          res.selected = selected;
          res.n_feasible = nfeas_k;
          res.status = status | uk.st_pf | (sc ? uk.st_sc : 0u);
          res.score_skip = sc ? uk.skip_sc : uk.skip;
          s_res[k] = res;
        }
        // the next round's speculation: pointers as they were before pod k's step
        if (lane > k && lane < nb) {
          ptr = s_snap[k * 64 + lane];
          cnode = ptr < u.K ? s_top[lane * KT + ptr] : -1;
          // a new node taken by pod k (the rescan's choice): lanes holding it step on
          bool conflict = selected >= 0 && idx < 0 && cnode == selected;
          while (conflict) {
            ptr++;
            cnode = ptr < u.K ? s_top[lane * KT + ptr] : -1;
            conflict = cnode >= 0 && sv_changed(s_cmask, cnode);
          }
        }
      }
      if (lane == 0) s_ctl[0] = ks < nb ? ks + 1 : nb;
      if (lane == 0) s_ctl[1] = nv_c;
      if (lane == 0) s_ctl[2] = ns_c;
    }
    __syncthreads();
    start = s_ctl[0];
    nv_c = s_ctl[1];
    ns_c = s_ctl[2];
  }
  if (tid == 0 && start < nb && a.tk_timeout) {   // cannot happen: each round commits >= 1 pod
    using G1 = __attribute__((address_space(1))) unsigned;
    __hip_atomic_store((G1*)a.tk_timeout, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- epilogue: rows, results, count tables, carry-out -----------------------------
  for (int x = tid; x < ns_c * SW; x += BLOCK) {
    const int s = x / SW, w = x - s * SW, node = s_clist[s];
    if (node < 0) continue;
    const int64_t val = s_vrow[(size_t)s_lastv[s] * kSvRow + w];
    if (w < 8 && (w & 1) && (w >> 1) < R) a.st.requested[(size_t)(w >> 1) * N + node] = val;
    else if (w == SL::NZC || w == SL::NZM) a.st.nonzero[(size_t)(w - SL::NZC) * N + node] = val;
    else if (w == SL::PODS) a.st.pod_count[node] = (int32_t)val;
  }
  for (int i = tid; i < nb; i += BLOCK) {
    a.placements[a.out0 + i] = s_res[i].selected;
    if (a.results) a.results[a.out0 + i] = s_res[i];
  }
  for (int i = tid; i < 2 * nb; i += BLOCK) a.pmax[i] = 0;   // ready for the next batch's phase 1
  if (tid == 0) {   // PodTopologySpread / InterPodAffinity count tables of the committed pods
    for (int k = 0; k < nb; k++) {
      const int sel = s_res[k].selected;
      if (sel < 0 || !(s_u[k].flags & 8u)) continue;
      const ksg_pod& p = s_pods[k];
      const int32_t* cw = s_prog + (p.commit - a.prog_lo);
      const int ns = *cw++;
      for (int i = 0; i < ns; i++) a.st.cnt[(size_t)cw[i] * N + sel] += 1;
      cw += ns;
      const int nt = *cw++;
      for (int i = 0; i < nt; i++) {
        const int t = cw[2 * i];
        const uint32_t lv = c.label_val[(size_t)c.tmpl_col[t] * N + sel];
        if (!lv) continue;
        a.st.tab[c.tmpl_off[t] + lv] += c.tmpl_kind[t] == KSG_TMPL_PREF ? cw[2 * i + 1] : 1;
        a.st.tmpl_total[t] += 1;
      }
    }
  }
  if (a.carry_out && wv == 0) {   // slots assumed onto in this batch, in slot order
    int base = 0;
    for (int b = 0; b < ns_c; b += 64) {
      const int s = b + lane;
      const bool t = s < ns_c && s_clist[s] >= 0 && s_vt[s_lastv[s]] >= 0;
      const uint64_t m = __ballot(t);
      if (t) a.carry_out[base + __popcll(m & ((1ull << lane) - 1))] = s_clist[s];
      base += __popcll(m);
    }
    if (lane == 0) *a.carry_out_n = base;
  }
}
