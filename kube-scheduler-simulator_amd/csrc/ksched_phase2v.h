// Phase 2, speculate-and-verify walk (KSG_BATCH_MODE=spec, the default for
// runs in its scope), included by ksched.hip after ksched_phase2t.h (it reuses
// the transposed walk's N32 column evaluation: TcPod / TcRow / tc_eval).
//
// The slot walk and the transposed walk both put one exact evaluation of a
// changed node on every pod's critical path.  On configs[1] about 97 % of the
// pods take their best UNCHANGED node (the first entry of the top set T_j
// outside the changed set D_j), which needs no evaluation at all: it follows
// from the top sets and from which nodes earlier pods took.  So the batch runs
// in rounds, each round from `start` (the first undecided pod):
//
//   S  speculate (wave 0, lane q = pod q): every pod takes its best unchanged
//      node.  Lane q keeps a pointer into T_q (staged in LDS) past every entry
//      already in D; per pod k one v_readlane gives d_k, the lanes whose
//      candidate is d_k step their pointer on (the next entry is read ahead;
//      one LDS read of the changed bitmap per step-on).  No evaluation on this
//      chain.  Every decision is published through an LDS progress counter, and
//      every lane's pointer is snapshotted per step (a rollback restores it).
//   V  verify, pipelined behind S (waves 1..7, lane = pod): each published
//      decision is a new row version of a node (its live columns + the pod's
//      deltas); a consumer wave fetches the row and evaluates the version for
//      all 64 pods at once (tc_eval's N32 Fit / BalancedAllocation, phase-1
//      records from the node-major copies) into a per-(slot, pod) column word.
//      Round 1 also evaluates the carried slots (the previous batch's nodes).
//      Column words of versions committed in earlier rounds stay valid, so a
//      round evaluates only its new versions.
//   A  aggregate (all waves): per pod, over every slot present at its turn, the
//      best live column key and the counters (phase-1 feasible, live, lost
//      TaintToleration / NodeAffinity maximum holders).
//   C  check (wave 0): each pod's exact decision from its counters, best column
//      and best unchanged key, exactly as the slot walk decides it.  The first
//      pod k* whose decision differs from the speculated one (or that needs the
//      renormalisation rescan) ends the round: pods before it are committed,
//      k*'s exact decision is applied (a new version of an existing slot, or a
//      new slot, evaluated as the next round's first item), the speculated
//      slots after it are dropped, and the next round speculates from k* + 1
//      with the pointers restored from k*'s snapshot.
//
// Every decision equals the sequential one: a pod's decision is committed only
// after verification against the state every earlier committed decision left,
// and k*'s decision is computed from that same verified state.  Results equal
// the slot walk's and the oracle's bit for bit.
//
// Scope (host: spec_candidate): N32 ranges, the compact Fit /
// BalancedAllocation profile, weighted totals < 2^27 (column words), <= 64-pod
// batches in the two-batch window.

constexpr int kSvWaves = 12;                  // wave 0 speculates (then verifies), 1..11 verify
constexpr int kSvSlots = 2 * 64;              // carried (<= previous batch) + this batch's
constexpr int kSvRow = SlotLayout<4>::STRIDE; // int64 words per LDS row
constexpr int kSvTotalBits = 27;
constexpr int kSvOwner = 2048;                // hashed owner table of the speculation's macro-steps

__device__ __forceinline__ bool sv_changed(const uint32_t* cm, int n) { return ((cm[n >> 5] >> (n & 31)) & 1u) != 0; }

// column word: total (27 bits) | live << 27 | phase-1 feasible << 28 | held the
// phase-1 TaintToleration maximum << 29 | ... NodeAffinity << 30 | present << 31
__device__ __forceinline__ uint32_t sv_word(int32_t total, bool live, bool p1f, bool ft, bool fa) {
  return ((uint32_t)total & ((1u << kSvTotalBits) - 1)) | (live ? 1u << 27 : 0u) | (p1f ? 1u << 28 : 0u) |
         (ft ? 1u << 29 : 0u) | (fa ? 1u << 30 : 0u) | (1u << 31);
}

// A queue entry of the verification: a row version to evaluate.
struct SvItem {
  int32_t node, slot, v;   // node, its slot, the version index (row stored at s_vrow[v])
  int32_t src;             // row source: a version index, or -1 (the node's live columns in global memory)
  int32_t t;               // the pod whose assume made the version (-1: none, the carried live row)
};

// One batch's walk (the body of both kernels below).
template <int BLOCK, bool MW = false>
__device__ __forceinline__ void spec_walk_batch(const BatchArgs& a) {
  using SL = SlotLayout<4>;
  constexpr int NW = BLOCK / 64;
  constexpr int SW = SL::W;
  static_assert(BLOCK == 64 * kSvWaves && SW == 16, "spec walk layout");
  extern __shared__ __attribute__((aligned(16))) int32_t s_dyn[];
  __shared__ ksg_profile s_prof;
  __shared__ __attribute__((aligned(16))) TcU s_u[64];
  __shared__ ksg_result s_res[64];
  __shared__ int32_t s_clist[kSvSlots];   // node of slot (-1: a hole, pod without a node)
  __shared__ int32_t s_lastv[kSvSlots];   // newest version of slot
  __shared__ int32_t s_vt[kSvSlots];      // pod whose assume made the version (-1: carried live row)
  __shared__ int32_t s_dec[64];           // pod's node (speculated, then committed)
  __shared__ uint64_t s_bu[64];           // pod's best unchanged key (0: none)
  __shared__ uint64_t s_best[64];         // aggregate: best live column key
  __shared__ uint32_t s_cnt[64];          // aggregate: p1 feasible | live << 8 | lost taint << 16 | lost aff << 24
  __shared__ uint8_t s_snap[64 * 64];     // [macro-step][pod] T pointers at the macro-step's start
  __shared__ uint8_t s_mstep[64];         // pod's macro-step in the current round
  __shared__ uint8_t s_dptr[64];          // pod's T pointer when it was decided
  __shared__ uint32_t s_owner[kSvOwner];  // lowest lane holding a node (hashed), 0xffffffff = none
  __shared__ SvItem s_item[64 + 1];       // a round's special items: carried slots / the correction
  __shared__ int32_t s_ctl[8];            // round: start, nv_c, ns_c, n_special; progress; next item
  __shared__ P1Stats s_p1[64];

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
  uint32_t* s_col = reinterpret_cast<uint32_t*>(s_vrow + (size_t)kSvSlots * kSvRow);   // [slot][64]
  int32_t* s_top = reinterpret_cast<int32_t*>(s_col + (size_t)kSvSlots * 64);         // [64][KT] nodes

#ifdef KSG_STAMPS
  unsigned long long st_acc[16] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif
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
  KSG_STAMP(8);   // the wait for this batch's phase 1 / top-k
  for (int i = tid; i < cm_words; i += BLOCK) s_cmask[i] = 0;
  for (int i = tid; i < kSvOwner; i += BLOCK) s_owner[i] = 0xffffffffu;
  {   // every staging load issued before the first LDS store
    constexpr int PI = (64 * POD_WORDS + BLOCK - 1) / BLOCK;
    int32_t pw[PI];
#pragma unroll
    for (int it = 0; it < PI; it++) {
      const int i = tid + it * BLOCK;
      pw[it] = i < nb * POD_WORDS ? reinterpret_cast<const int32_t*>(a.pods + a.b0)[i] : 0;
    }
#pragma unroll
    for (int it = 0; it < PI; it++) {
      const int i = tid + it * BLOCK;
      if (i < nb * POD_WORDS) reinterpret_cast<int32_t*>(s_pods)[i] = pw[it];
    }
  }
  for (int i0 = 0; i0 < a.prog_len; i0 += 4 * BLOCK) {
    int32_t g[4];
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int i = i0 + tid + it * BLOCK;
      g[it] = i < a.prog_len ? a.prog[a.prog_lo + i] : 0;
    }
#pragma unroll
    for (int it = 0; it < 4; it++) {
      const int i = i0 + tid + it * BLOCK;
      if (i < a.prog_len) s_prog[i] = g[it];
    }
  }
  for (int i = tid; i < (int)(sizeof(ksg_profile) / 4); i += BLOCK)
    reinterpret_cast<int32_t*>(&s_prof)[i] = reinterpret_cast<const int32_t*>(a.prof)[i];
  bool fit_filter_on = false;
  for (int kf = 0; kf < a.prof->n_filter; kf++) fit_filter_on |= a.prof->filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  {   // T as node indices, [pod][KT]: two keys per 16-byte load, every load issued
      // before the first store; entries past a pod's K are never read (every
      // reader bounds its pointer by K), so they are converted unchecked
    const int KP = (KT + 1) >> 1;   // key pairs per row
    constexpr int TI = (64 * kSvSlots / 2 + BLOCK - 1) / BLOCK;
    ulonglong2 kp[TI];
#pragma unroll
    for (int it = 0; it < TI; it++) {
      const int x = tid + it * BLOCK, q = x / KP, i = 2 * (x - q * KP);
      const uint64_t* tp = a.top + (size_t)q * KSG_BATCH_MAX + i;
      if (x >= nb * KP) kp[it] = ulonglong2{0, 0};
      else if (a.tk_sc) kp[it] = ulonglong2{ld_sc(tp), ld_sc(tp + 1)};   // top-k's sc0 sc1 hand-off
      else kp[it] = *reinterpret_cast<const ulonglong2*>(tp);
    }
#pragma unroll
    for (int it = 0; it < TI; it++) {
      const int x = tid + it * BLOCK, q = x / KP, i = 2 * (x - q * KP);
      if (x < nb * KP) {
        s_top[q * KT + i] = key_node(kp[it].x);
        if (i + 1 < KT) s_top[q * KT + i + 1] = key_node(kp[it].y);
      }
    }
  }
  if (tid < nb * (int)(sizeof(P1Stats) / 4)) {   // the pods' phase-1 statistics, read once
    const int32_t* src = reinterpret_cast<const int32_t*>(a.p1) + tid;
    reinterpret_cast<int32_t*>(s_p1)[tid] = a.tk_sc ? ld_sc(src) : *src;
  }
  KSG_STAMP(9);   // staging loads issued and stored
  // carried slots: slot t = version t = carried node t, evaluated as round 1's
  // special items (their rows come from global memory)
  const int nc0 = a.carry ? *a.carry_n : 0;
  if (tid < 64) {
    const int d = a.carry && tid < nc0 ? a.carry[tid] : 0;
    if (tid < nc0) {
      s_clist[tid] = d;
      s_lastv[tid] = tid;
      s_vt[tid] = -1;
      s_item[tid] = SvItem{d, tid, tid, -1, -1};
    }
  }
  __syncthreads();
  const ksg_profile& prof = s_prof;
  const TcProf cm = tc_prof(cm_prof(prof));
  if (tid < nc0) atomicOr(&s_cmask[s_clist[tid] >> 5], 1u << (s_clist[tid] & 31));
  if (wv == 0 && lane < nb) {
    const bool ipa_filter = ipa_in_filter(prof);
    const bool ipa_score = ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) != 0;
    const ksg_pod& p = s_pods[lane];
    const P1Stats s1 = s_p1[lane];
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
  if (tid == 0) {
    s_ctl[0] = 0;     // start
    s_ctl[1] = nc0;   // committed versions
    s_ctl[2] = nc0;   // committed slots
    s_ctl[3] = nc0;   // special items of round 1: the carried slots
    s_ctl[4] = 0;     // progress: speculation steps published
    s_ctl[6] = 0;     // next verification item to take
  }
  __syncthreads();
  // initial pointers: T_q's first entry outside the carried nodes (wave w: pods w, w + NW, ...)
  for (int q = wv; q < nb; q += NW) {
    const int K = s_u[q].K;
    int ptr = K;
    for (int b = 0; b < K && ptr == K; b += 64) {
      const int i = b + lane;
      const int n = i < K ? s_top[q * KT + i] : -1;
      const uint64_t m = __ballot(i < K && !sv_changed(s_cmask, n));
      if (m) ptr = b + __builtin_ctzll(m);
    }
    if (lane == 0) s_dptr[q] = (uint8_t)ptr;   // the round-1 pointers
  }
  __syncthreads();

  // pod t's row delta word `w` (the assume: requested += req, nonzero, pod count)
  auto delta_word = [&](const TcU& u, int w) -> int64_t {
    const int rl = (w >> 1) & 3;
    const int64_t req_l = rl == 0 ? u.req[0] : rl == 1 ? u.req[1] : rl == 2 ? u.req[2] : u.req[3];
    return w < 8 ? ((w & 1) ? req_l : 0) : w == SL::NZC ? u.nzc : w == SL::NZM ? u.nzm : w == SL::PODS ? 1 : 0;
  };
  // lane q's pod (consumer waves evaluate every version for every pod)
  const int qq = lane < nb ? lane : 0;
  const TcPod hp = tc_pod(s_pods[qq], prof, s_p1[qq], fit_filter_on, R);
  // Evaluate one row version for every pod into its slot's column words (a
  // consumer wave).  Pods after t see it; a new slot is absent for the pods up
  // to t; a re-choice leaves the earlier pods their previous version's words.
  // Split in two so that the next item's loads are in flight while this one
  // is evaluated: issue() starts the loads, finish() evaluates.
  struct Pending {
    SvItem it;
    uint64_t x;    // pod lane's phase-1 record at the node
    int32_t st;    // pod lane's weight x ImageLocality at the node (the static part after finish's terms)
    int64_t wd;    // row word `lane` (lanes < SW) before the pod's delta
  };
  auto issue = [&](const SvItem& it) -> Pending {
    Pending p{it, 0, 0, 0};
    if (it.node < 0) return p;
    if (a.inject_walk_err && lane == 0 && it.node >= 0) {   // tests: the report path below, without a bad load
      using G1 = __attribute__((address_space(1))) unsigned;
      __hip_atomic_store((G1*)a.walk_err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (it.node >= N) {   // cannot happen; never load through it (reported as code 3)
      p.it.node = -1;
      if (lane == 0) {
        using G1 = __attribute__((address_space(1))) unsigned;
        __hip_atomic_store((G1*)a.walk_err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return p;
    }
    // the node-major copies phase 1 wrote: record and weight x ImageLocality
    p.x = a.rect[(size_t)it.node * 64 + lane];
    p.st = a.imgt[(size_t)it.node * 64 + lane];
    const int wl = lane < SW ? lane : 0;
    p.wd = it.src >= 0 ? s_vrow[(size_t)it.src * kSvRow + wl]
                       : slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, wl, R, it.node), wl, R);
    return p;
  };
  auto finish = [&](const Pending& p) {
    const SvItem& it = p.it;
    if (it.node < 0) return;
    if (lane < SW) s_vrow[(size_t)it.v * kSvRow + lane] = p.wd + (it.t >= 0 ? delta_word(s_u[it.t], lane) : 0);
    int64_t w[SW];
    {
      const int4* src = reinterpret_cast<const int4*>(s_vrow + (size_t)it.v * kSvRow);
#pragma unroll
      for (int k = 0; k < SW / 2; k++) reinterpret_cast<int4*>(w)[k] = src[k];
    }
    const TcRow row = tc_row<MW>(cm, w);
    const bool p1f = (p.x >> 63) != 0;
    const bool ft = p1f && (int32_t)((p.x >> 48) & 0xff) == hp.mt;
    const bool fa = p1f && (int32_t)((p.x >> 32) & 0xffff) == hp.ma;
    // the static part of the total: top-k's total_score terms under the phase-1
    // maxima (TaintToleration 100 - 100 rt / mt, NodeAffinity 100 ra / ma, floor
    // divisions; the same qdiv32 as the transposed walk)
    const int32_t rt = (int32_t)((p.x >> 48) & 0xff), ra = (int32_t)((p.x >> 32) & 0xffff);
    const int32_t nt = hp.mt != 0 ? 100 - qdiv32(100 * rt, hp.mt, hp.inv_mt) : 100;
    const int32_t na = hp.ma != 0 ? qdiv32(100 * ra, hp.ma, hp.inv_ma) : ra;
    const int32_t stat = p.st + hp.wt * nt + hp.wa * na;
    int32_t fb = 0;
    const bool live = tc_eval<MW>(cm, hp, row, fb) && p1f;
    if (lane > it.t) s_col[it.slot * 64 + lane] = sv_word(stat + fb, live, p1f, ft, fa);
    else if (it.src < 0) s_col[it.slot * 64 + lane] = 0u;
  };

  // wave 0's speculation state: lane q's pointer into T_q, its node (-1: none)
  // and the entry after it (read ahead: a step-on costs one LDS round trip)
  int ptr = 0, cnode = -1, nnode = -1;
  if (wv == 0 && lane < nb) {
    ptr = s_dptr[lane];
    const int K = s_u[lane].K;
    cnode = ptr < K ? s_top[lane * KT + ptr] : -1;
    nnode = ptr + 1 < K ? s_top[lane * KT + ptr + 1] : -1;
  }
  int start = 0, nv_c = nc0, ns_c = nc0, nspecial = nc0;
  int guard = 0;
  KSG_STAMP(0);
  while (start < nb && guard++ <= nb) {
#ifdef KSG_STAMPS
    if (tid == 0) st_acc[15] += 1;   // rounds
#endif
    if (wv == 0) {
      // ---- S: speculate, publishing each step ---------------------------------------
      // (the chain's wave issues first where it shares a SIMD with a consumer)
      __builtin_amdgcn_s_setprio(3);
      if (lane >= start && lane < nb) {
        s_best[lane] = 0;
        s_cnt[lane] = 0;
      }
      const int Kq = lane < nb ? s_u[lane].K : 0;
      // Macro-steps: every undecided pod from `cur` on holds a free candidate;
      // the pods up to the first one whose candidate an earlier one also holds
      // (found through a hashed table of the lowest lane per node: ds_min) take
      // their candidates at once, exactly as the one-pod steps would (none of
      // them conflicts with an earlier one); then the later pods whose
      // candidate was taken step on.  Pointer snapshots per macro-step; a
      // rollback restores the one of k*'s macro-step and re-validates.
      int mi = 0;
      for (int cur = start; cur < nb; mi++) {
        s_snap[mi * 64 + lane] = (uint8_t)ptr;
        const bool act = lane >= cur && lane < nb && cnode >= 0;
        const int hsh = cnode & (kSvOwner - 1);
        if (act) atomicMin(&s_owner[hsh], (unsigned)lane);
        // (one wave: the LDS executes its DS instructions in order, so this read sees every lane's min)
        const unsigned o = act ? s_owner[hsh] : (unsigned)lane;
        const uint64_t dup = __ballot(act && o != (unsigned)lane);
        const int f = dup ? __builtin_ctzll(dup) : nb;
#ifdef KSG_STAMPS
        if (tid == 0) { st_acc[14] += f - cur; st_acc[12] += 1; }   // steps, macro-steps
#endif
        if (lane >= cur && lane < f) {   // the run: decided
          s_dptr[lane] = (uint8_t)ptr;
          s_mstep[lane] = (uint8_t)mi;
          if (cnode >= 0) atomicOr(&s_cmask[cnode >> 5], 1u << (cnode & 31));
        }
        if (act) s_owner[hsh] = 0xffffffffu;
        if (lane == 0) {   // publish (in-order DS: a consumer that sees it sees s_dptr / s_mstep)
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          __hip_atomic_store(&s_ctl[4], f - start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // later pods whose candidate the run took (the owner prefilter has no
        // false negatives; the bitmap decides, hashing collisions included)
        bool conflict = lane >= f && lane < nb && cnode >= 0 && o < (unsigned)f && sv_changed(s_cmask, cnode);
        while (__ballot(conflict)) {
#ifdef KSG_STAMPS
          if (tid == 0) st_acc[13] += 1;   // step-on iterations
#endif
          if (conflict) {
            ptr++;
            cnode = nnode;
            nnode = ptr + 1 < Kq ? s_top[lane * KT + ptr + 1] : -1;
            conflict = cnode >= 0 && sv_changed(s_cmask, cnode);
          }
        }
        cur = f;
      }
      __builtin_amdgcn_s_setprio(0);
      KSG_STAMP(1);
    }
    {
      // ---- V: verify behind the speculation (waves 1.., and wave 0 once S is done) ------
      // items are taken in order from an LDS counter (load balance across the
      // waves); items [0, nspecial): s_item (carried slots / the correction); then
      // pod k = start + (i - nspecial) once the speculation published it (a
      // hole, node -1, when the pod took no node).  take(): 1 taken, 0 not
      // published yet (only when !wait), -1 past the end.
      auto take = [&](int i, bool wait, SvItem& it) -> int {
        it = SvItem{-1, 0, 0, -1, -1};   // (a hole unless filled below: never issue() an unset item)
        if (i < nspecial) {
          it = s_item[i];
          return 1;
        }
        const int k = start + (i - nspecial);
        if (k >= nb) return -1;
        // (bounded: every step is published, the bound only keeps a fault from hanging the launch)
        for (unsigned spins = 0;
             __hip_atomic_load(&s_ctl[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= k - start; spins++) {
          if (!wait) return 0;
          if (spins >= (1u << 24)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int sl = ns_c + (k - start), v = nv_c + (k - start);
        const int pk = s_dptr[k];
        const int d = pk < s_u[k].K ? s_top[k * KT + pk] : -1;   // pod k's speculated node
        if (lane == 0) {
          s_dec[k] = d;
          s_clist[sl] = d;
          s_lastv[sl] = v;
          s_vt[v] = k;
          const uint64_t* tp = a.top + (size_t)k * KSG_BATCH_MAX + pk;
          s_bu[k] = d < 0 ? 0 : a.tk_sc ? ld_sc(tp) : *tp;
        }
        it = SvItem{d, sl, v, -1, k};
        return 1;
      };
      auto grab = [&]() -> int {
        int i = 0;
        if (lane == 0) i = atomicAdd(&s_ctl[6], 1);
        return __builtin_amdgcn_readfirstlane(i);
      };
      SvItem ia, ib;
      int xa = grab();
      int ra = take(xa, true, ia);
      Pending pa = issue(ia), pb = issue(SvItem{-1, 0, 0, -1, -1});
      while (ra > 0) {
        const int xb = grab();
        int rb = take(xb, false, ib);
        if (rb > 0) pb = issue(ib);
        finish(pa);
        if (rb == 0) {
          rb = take(xb, true, ib);
          if (rb > 0) pb = issue(ib);
        }
        if (rb < 0) break;
        xa = grab();
        ra = take(xa, false, ia);
        if (ra > 0) pa = issue(ia);
        finish(pb);
        if (ra == 0) {
          ra = take(xa, true, ia);
          if (ra > 0) pa = issue(ia);
        }
      }
      KSG_STAMP(2);
    }
    __syncthreads();
    KSG_STAMP(3);
    // ---- A: aggregate every slot present at each pod's turn (wave w: slots w, w + NW, ...)
    {
      const int ns = ns_c + (nb - start);
      const bool mine = lane >= start && lane < nb;
      uint32_t dc = 0;   // this wave's slots, in registers; one LDS atomic per pod at the end
      uint64_t bk = 0;
      for (int s = wv; s < ns; s += NW) {
        const int node = s_clist[s];
        if (node < 0) continue;
        const uint32_t e = s_col[s * 64 + lane];
        const bool pres = (e >> 31) != 0;
        const bool live = pres && ((e >> 27) & 1u), p1f = pres && ((e >> 28) & 1u);
        const bool ft = (e >> 29) & 1u, fa = (e >> 30) & 1u;
        dc += (p1f ? 1u : 0u) + (live ? 1u << 8 : 0u) + (p1f && !live && ft ? 1u << 16 : 0u) +
              (p1f && !live && fa ? 1u << 24 : 0u);
        const uint64_t key = live ? argmax_key((int64_t)(e & ((1u << kSvTotalBits) - 1)), node) : 0;
        bk = key > bk ? key : bk;
      }
      if (mine && dc) atomicAdd(&s_cnt[lane], dc);
      if (mine && bk) atomicMax(reinterpret_cast<unsigned long long*>(&s_best[lane]), (unsigned long long)bk);
    }
    __syncthreads();
    KSG_STAMP(4);
    // ---- C: check + commit (wave 0) ------------------------------------------------
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
      nspecial = 0;
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
          const TcPod hk = tc_pod(p, prof, s_p1[k], fit_filter_on, R);
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
            if (!tc_eval<MW>(cm, hk, tc_row<MW>(cm, w), fb)) return 0;
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
        if (selected >= 0) {   // the corrected version: the next round's first item
          const int s = idx >= 0 ? idx : ns_c, v = nv_c;
          if (lane == 0) {
            s_item[0] = SvItem{selected, s, v, idx >= 0 ? s_lastv[idx] : -1, k};
            if (idx < 0) {
              s_clist[s] = selected;
              s_cmask[selected >> 5] |= 1u << (selected & 31);
            }
            s_lastv[s] = v;
            s_vt[v] = k;
          }
          nspecial = 1;
          nv_c += 1;
          if (idx < 0) ns_c += 1;
        }
        if (lane == 0) {
          s_dec[k] = selected;
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
          ptr = s_snap[s_mstep[k] * 64 + lane];   // at the start of k's macro-step
          cnode = ptr < u.K ? s_top[lane * KT + ptr] : -1;
          nnode = ptr + 1 < u.K ? s_top[lane * KT + ptr + 1] : -1;
          // re-validate: nodes the committed pods of that macro-step took, and a
          // new node taken by pod k (the rescan's choice), are stepped over
          bool conflict = cnode >= 0 && sv_changed(s_cmask, cnode);
          while (conflict) {
            ptr++;
            cnode = nnode;
            nnode = ptr + 1 < u.K ? s_top[lane * KT + ptr + 1] : -1;
            conflict = cnode >= 0 && sv_changed(s_cmask, cnode);
          }
        }
      }
      if (lane == 0) {
        s_ctl[0] = ks < nb ? ks + 1 : nb;
        s_ctl[1] = nv_c;
        s_ctl[2] = ns_c;
        s_ctl[3] = nspecial;
        s_ctl[4] = 0;
        s_ctl[6] = 0;
      }
    }
    KSG_STAMP(5);
    __syncthreads();
    KSG_STAMP(6);
    start = s_ctl[0];
    nv_c = s_ctl[1];
    ns_c = s_ctl[2];
    nspecial = s_ctl[3];
  }
  if (tid == 0 && start < nb) {   // cannot happen: each round commits >= 1 pod
    using G1 = __attribute__((address_space(1))) unsigned;
    __hip_atomic_store((G1*)a.walk_err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- epilogue: rows, results, count tables, carry-out -----------------------------
  // (a correction left as the last round's item has its row written here)
  if (nspecial && wv == 0) {
    const SvItem it = s_item[0];
    if (lane < SW) {
      int64_t wd = it.src >= 0 ? s_vrow[(size_t)it.src * kSvRow + lane]
                               : slot_word_value<4, true>(slot_word_fetch<4, true>(c, a.st, lane, R, it.node), lane, R);
      wd += delta_word(s_u[it.t], lane);
      s_vrow[(size_t)it.v * kSvRow + lane] = wd;
    }
  }
  __syncthreads();
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
  uint64_t cmt = 0;   // pods with count-table updates (PodTopologySpread / InterPodAffinity selectors)
  if (wv == 0) cmt = __ballot(lane < nb && s_res[lane].selected >= 0 && (s_u[lane].flags & 8u));
  if (tid == 0 && cmt) {
    for (int k = 0; k < nb; k++) {
      if (!((cmt >> k) & 1ull)) continue;
      const int sel = s_res[k].selected;
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
  KSG_STAMP(7);
#ifdef KSG_STAMPS
  if (tid == 0 && a.stamps)
    for (int i = 0; i < 16; i++) atomicAdd(&a.stamps[i], st_acc[i]);
#endif
}

// One launch per batch (stream-ordered runs, the counter passes).
template <int BLOCK, bool MW = false>
__global__ __launch_bounds__(BLOCK) void ksg_batch_phase2v(BatchArgs a) {
  spec_walk_batch<BLOCK, MW>(a);
}

// The persistent walk (round 6): one launch walks every batch of the run, so
// the single-workgroup walk no longer pays a dispatch, its kernel-boundary
// cache operations and an event between batches (a 6.6 us median gap per
// 64-pod batch on the headline, profiles/r6).  Batch b's arguments come from
// the host's table; its top-k hand-off is the same flag poll.  After each
// batch every wave drains its stores, one lane writes the XCD's L2 back (agent
// release: the node state, the zeroed maxima and the carry that phase 1 of
// batch b + 2 reads from other XCDs) and stores b + 1 into the host-visible
// counter; the host launches phase 1 / top-k of batch b + 2 once it reads it
// (their dispatch acquires).  A timed-out hand-off or a broken invariant ends
// the loop (the host reports it).
struct SpecRun {
  const int32_t* btab;   // [nbatch][6]: b0, out0, nb, prog_lo, prog_len, k_extra
  int32_t nbatch;
  uint64_t* rec[2];
  int32_t* img[2];
  uint64_t* rect[2];
  int32_t* imgt[2];
  int32_t* pmax[2];
  P1Stats* p1[2];
  uint64_t* top[2];
  int32_t* carry;        // [2][KSG_BATCH_MAX]
  int32_t* carry_n;      // [2]
  unsigned* done;        // batches walked (pinned host memory, the device address)
};

template <int BLOCK, bool MW = false>
__global__ __launch_bounds__(BLOCK) void ksg_batch_phase2v_run(BatchArgs base, SpecRun r) {
  __shared__ int s_stop;
  using G1 = __attribute__((address_space(1))) unsigned;
  for (int bi = 0; bi < r.nbatch; bi++) {
    BatchArgs a = base;
    const int32_t* d = r.btab + 6 * bi;
    a.b0 = d[0];
    a.out0 = d[1];
    a.nb = d[2];
    a.prog_lo = d[3];
    a.prog_len = d[4];
    a.k_extra = d[5];
    const int par = bi & 1;
    a.rec = r.rec[par];
    a.img = r.img[par];
    a.rect = r.rect[par];
    a.imgt = r.imgt[par];
    a.pmax = r.pmax[par];
    a.p1 = r.p1[par];
    a.top = r.top[par];
    a.carry = r.carry + (par ^ 1) * KSG_BATCH_MAX;
    a.carry_n = r.carry_n + (par ^ 1);
    a.carry_out = r.carry + par * KSG_BATCH_MAX;
    a.carry_out_n = r.carry_n + par;
    a.tk_seq = (unsigned)bi + 1;
    spec_walk_batch<BLOCK, MW>(a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores performed
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store((G1*)r.done, (unsigned)bi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_stop = (__hip_atomic_load((G1*)base.tk_timeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                __hip_atomic_load((G1*)base.walk_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
    }
    __syncthreads();
    if (s_stop) break;
  }
}
