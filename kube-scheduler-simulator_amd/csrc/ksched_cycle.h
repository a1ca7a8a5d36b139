// The per-cycle evaluation (ksg_eval's fast path, the Go shim's one call per
// scheduling cycle, wrappedplugin.go:388-548), included by ksched_dev.h inside
// namespace ksk.
//
// One launch of G = ceil(N / (64 KN)) one-wave workgroups, all co-resident,
// KN nodes per lane (lane l of workgroup g owns nodes (k G + g) 64 + l),
// results written straight into the pinned, fine-grained host block the
// caller reads in place (ksg_eval_view).  The round-5 form is built around
// the latency chain of one wave, not around throughput:
//
//   entry      the kernel arguments carry everything the wave needs: the node
//              column pointers, the pod record, the profile facts the host
//              derived for this pod (filter order as nibbles, the filters and
//              scores that run, weights, the compact Fit / BalancedAllocation
//              form) and up to kCycBlob words of the pod's programs.  Every
//              64-byte line of the scalar part is touched by one s_load at
//              entry (one miss latency for all of them, instead of one per
//              use site deep in the evaluation: round 4's kernel waited on
//              ~60 scattered kernel-argument loads); the programs are copied
//              to LDS by vector loads issued beside them.
//   prefetch   every node column the evaluation can touch is loaded at once:
//              the resource columns, the unschedulable byte, the first
//              kCycLab label columns, kCycTnt taint slots and (scoring
//              ImageLocality) kCycImg image slots into registers, the taint
//              effect table into LDS; a deeper column falls back to a global
//              load.
//   evaluate   every filter the pod runs is evaluated independently (no
//              first-rejection chain of dependent loads), then the status word
//              is the first rejection in profile order; raw scores of a
//              feasible node.
//   exchange   the wave's feasible count, TaintToleration / NodeAffinity
//              maxima and lowest feasible index (DPP reductions) go to its
//              own slot; grid exchange on per-workgroup flags tagged with the
//              call's sequence number (agent-scope stores and loads, no reset
//              between calls); every workgroup folds the G slots.
//   rows       status words and raw rows (2, 4 or 8 bytes) to the host block
//              (SYS, the default: system-scope stores and a vmcnt wait; else
//              plain stores and __threadfence_system); the normalised rows
//              and the totals are not stored (round 6: the host derives the
//              normalised TaintToleration / NodeAffinity values from the raw
//              rows and the maxima of the result line; nothing reads the
//              totals); the
//              selectHost keys and error bits fold into device slots by
//              atomics, and the last workgroup to arrive stores the result
//              line and its done word: the host polls one word.
//
// ksg_cycle_server<KN, SYS> is the same evaluation as a persistent kernel
// (KSG_CYCLE_SERVER=1): the node columns are loaded once and stay in
// registers / LDS, and each cycle's call (CycCall + programs) arrives in a
// pinned host mailbox the workgroups poll, so a cycle pays neither a launch
// nor the entry latencies.  It leaves on a stop request, after kSrvIdle of
// idleness (the host never calls a server idle for more than 0.05 s: it
// restarts it instead, so a call never races the idle exit), or when an
// exchange times out, so every wave always ends.
//
// The evaluation is eval_node_src's arithmetic (same helpers: untolerated_slot,
// na_required_match, fit_filter, fit_ba_cm / fit_score / ba_score,
// image_score, taint_score, na_pref_score) on a prefetched node source, and
// the normalisation is total_score's (untolerated_slot / taint_score /
// image_score restated on the prefetched registers: pnode_taints,
// pnode_image_score): results equal ksg_capture_eval +
// ksg_capture_norm (nb = 1, nothing assumed) bit for bit.

constexpr int kCycBlob = 256;    // program words carried in the kernel arguments
constexpr int kCycLab = 8;       // label columns prefetched into LDS rows
constexpr int kCycTnt = 8;       // taint slots prefetched into registers
constexpr int kCycImg = 8;       // image slots prefetched into registers (ImageLocality pods)
constexpr int kCycEff = 4096;    // taint-effect bytes staged in LDS
constexpr int kCycMaxKN = 4;     // nodes per lane
constexpr unsigned long long kSrvIdle = 10000000ull;   // server: 0.1 s of the 100 MHz real-time clock (the
                                                      // host restarts a server idle for 0.05 s).  Short: a
                                                      // running server holds back every device-wide
                                                      // synchronisation of the process (hipFree) until it
                                                      // leaves

// What does not change between calls on a loaded context.
struct CycStatic {
  DevCluster c;
  int64_t* requested;
  int64_t* nonzero;
  int32_t* pod_count;
  const uint32_t* used_ports;
  unsigned* flags;                   // [G][32]: workgroup g's exchange line (cyc_arrive) at [g * 32]
  unsigned* timeout;                 // sticky: an exchange poll gave up (reported to the host)
  unsigned* arrive;                  // completion counter (monotonic; a multiple of G between calls)
  unsigned long long* key;           // the running call's best selectHost key (zero between calls)
  unsigned* errw;                    // its error bits (zero between calls)
  unsigned long long* stamps;        // KSG_STAMPS builds: per-segment cycle sums of workgroup 0
};

// One call: the pod, the profile facts the host derived for it, the deferred
// assume of the previous pod, a staged append, where the rows go.
struct CycCall {
  const int32_t* gprog;              // the program pool as the kernel sees it (node_set; programs not inline)
  ksg_pod pod;
  uint64_t forder;                   // filter plugins in profile order, 4 bits each
  int32_t n_filter;
  uint32_t fmask;                    // plugins of the order that run their Filter for this pod
  uint32_t smask;                    // plugins whose Score runs for this pod (PodView::smask)
  int32_t w_fit, w_ba, w_img, w_t, w_a;
  uint32_t fit_ignored;
  int32_t cm_fast, cm_least;
  int64_t cm_wc, cm_wm;
  float cm_inv_ws, cm_inv_wc, cm_inv_wm;
  const ksg_profile* gprof;          // device copy (the generic Fit / BalancedAllocation forms)
  int32_t cm_node;                   // the deferred assume: -1 none; else its owner lane adds it first
  int64_t cm_req[KSG_MAX_RES];
  int64_t cm_nz_cpu, cm_nz_mem;
  ksg_pod* wpods;                    // a staged append of this pod (workgroup 0 writes it); null: none
  int32_t* wprog;
  const int32_t* sprog;
  int64_t slen;
  int32_t n_rows, es, kn;
  uint64_t rows;                     // score row q's plugin in bits 4q..4q+3
  uint32_t* h_fs;                    // [N]          (fine-grained pinned host memory, device addresses)
  char* h_raw;                       // [n_rows][N]  (the normalised rows and the totals are not stored: the
                                     // host derives them from these and the maxima in h_stats)
  int32_t* h_stats;                  // [8] nfeas, max taint, max node affinity, max (N - n), best key (2 words),
                                     // error bits, done (= seq; stored last, by the last workgroup)
  unsigned seq;
  int32_t op;                        // server mailbox: 0 evaluate, 1 stop
  const int32_t* bsrc;               // the programs when they are not inline
  int32_t blob_len;
  int32_t pad_;
};

// The launch arguments of ksg_eval_cycle: scalar part first (warmed line by
// line at entry), the program words last (copied to LDS by vector loads).
struct CycArgs {
  CycStatic s;
  CycCall k;
  int32_t blob[kCycBlob];
};

// The persistent server's mailbox (pinned host memory): the host writes the
// call and its programs, then `seq` (x86 stores are ordered; the server reads
// seq, then the rest, with system-scope loads).
struct SrvMailbox {
  unsigned seq;
  unsigned pad_[15];
  CycCall k;
  int32_t blob[KSG_BLOB_MAX];
};
struct SrvArgs {
  CycStatic s;
  const SrvMailbox* mb;              // device address of the mailbox
  CycCall* d_call;                   // device copy of the current call (workgroup 0 relays it) ...
  int32_t* d_blob;                   // ... and of its programs
  unsigned* d_go;                    // 128-byte line: the relayed call's sequence number
  unsigned last;                     // the last sequence number served before this launch
  int32_t want_img;                  // the profile scores ImageLocality: keep the image slots
  int32_t direct;                    // 1: the mailbox is fine-grained device memory: every workgroup polls
                                     // it and reads the call itself (no relay)
};

// The node a lane evaluates, its columns prefetched: the first kCycLab label
// columns in an LDS row of the lane (labels are looked up by a column the
// pod's programs name at run time: an indexed register array would live in
// scratch), the first kCycTnt taint and kCycImg image slots in registers
// (read only with constant indices, by pnode_taints / pnode_image_score),
// global memory beyond them; taint effects from the LDS copy when the
// vocabulary fits.
#define KSG_G1 __attribute__((address_space(1)))
#define KSG_L3 __attribute__((address_space(3)))
struct PNode {
  // the columns beyond the prefetched ones (values, not a pointer to the
  // launch arguments: taking the arguments' address copies them to scratch)
  const KSG_G1 uint32_t* label_val;
  const KSG_G1 int64_t* label_num;
  const KSG_G1 uint8_t* label_num_ok;
  const KSG_G1 uint32_t* taints;
  const KSG_G1 uint8_t* taint_effect;
  const KSG_G1 uint32_t* images;
  size_t N;
  int n;
  const KSG_L3 uint32_t* lab;   // this lane's prefetched labels: lab[q * 64]
  uint32_t tnt[kCycTnt], img[kCycImg];
  bool uns;
  bool eff_lds;
  const KSG_L3 uint8_t* eff;
  __device__ __forceinline__ uint32_t label(int col) const {
    return col < kCycLab ? lab[col * 64] : label_val[(size_t)col * N + n];
  }
  __device__ __forceinline__ bool num(int col, int64_t& x) const {
    const size_t k = (size_t)col * N + n;
    if (!label_num_ok[k]) return false;
    x = label_num[k];
    return true;
  }
  __device__ __forceinline__ uint8_t effect(uint32_t vid) const { return eff_lds ? eff[vid] : taint_effect[vid]; }
  __device__ __forceinline__ bool unsched() const { return uns; }
};

// untolerated_slot + taint_score on a prefetched node (the same walks: slots in
// order until the 0 terminator), the register slots with constant indices.
__device__ __forceinline__ void pnode_taints(const PNode& x, int T, const int32_t* tolf, const int32_t* tolp,
                                             bool want_slot, bool want_score, int& slot, int64_t& score) {
  slot = -1;
  score = 0;
  bool end = false;
  auto one = [&](int s, uint32_t id) {
    if (end || s >= T || !id) {
      end = true;
      return;
    }
    const uint32_t vid = id - 1;
    const uint8_t e = x.effect(vid);
    if (want_slot && slot < 0 && (e == KSG_EFFECT_NO_SCHEDULE || e == KSG_EFFECT_NO_EXECUTE) && !tol_bit(tolf, vid))
      slot = s;
    if (want_score && e == KSG_EFFECT_PREFER_NO_SCHEDULE) score += !tol_bit(tolp, vid);
  };
#pragma unroll
  for (int s = 0; s < kCycTnt; s++) one(s, x.tnt[s]);
  for (int s = kCycTnt; s < T && !end; s++) one(s, x.taints[(size_t)s * x.N + x.n]);
}

// image_score on a prefetched node: per container of the pod, the node's
// ascending image slots until the id is reached or passed.
__device__ __forceinline__ int64_t pnode_image_score(const PNode& x, int I, const int32_t* P, int img,
                                                     int n_containers) {
  int64_t sum = 0;
  if (img >= 0) {
    const int32_t* w = P + img;
    const int cnt = *w++;
    for (int i = 0; i < cnt; i++, w += 3) {
      const uint32_t id = (uint32_t)w[0];
      const int64_t contrib = ld64(w + 1);
      bool done = false;
#pragma unroll
      for (int s = 0; s < kCycImg; s++) {
        const uint32_t v = x.img[s];
        if (!done && s < I) {
          if (!v || v > id) done = true;
          else if (v == id) { sum += contrib; done = true; }
        } else {
          done = true;
        }
      }
      if (!done)
        for (int s = kCycImg; s < I; s++) {
          const uint32_t v = x.images[(size_t)s * x.N + x.n];
          if (!v || v > id) break;
          if (v == id) { sum += contrib; break; }
        }
    }
  }
  const int64_t mb = 1024 * 1024, minT = 23 * mb;
  const int64_t mx = 1000 * mb * (int64_t)n_containers;
  if (sum < minT) sum = minT;
  else if (sum > mx) sum = mx;
  return div_small(100 * (sum - minT), mx - minT);
}

#ifdef KSG_STAMPS
#define KSG_YSTAMP(seg)                                                       \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();               \
    if (blockIdx.x == 0) { y_acc[seg] += _t - y_last; y_last = _t; }          \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#else
#define KSG_YSTAMP(seg) do {} while (0)
#endif

// One scalar load per 64-byte line of CycArgs' scalar part (the first 768
// bytes of the argument segment), all in flight together and drained by one
// wait inside the same statement (a load may not be left pending into a
// register the compiler reuses): every later scalar read of an argument hits
// the scalar cache.  Loads only.
__device__ __forceinline__ void cyc_warm_args() {
  auto k = __builtin_amdgcn_kernarg_segment_ptr();
  uint32_t d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11;
  asm volatile(
      "s_load_dword %0, %12, 0x0\n\t"
      "s_load_dword %1, %12, 0x40\n\t"
      "s_load_dword %2, %12, 0x80\n\t"
      "s_load_dword %3, %12, 0xc0\n\t"
      "s_load_dword %4, %12, 0x100\n\t"
      "s_load_dword %5, %12, 0x140\n\t"
      "s_load_dword %6, %12, 0x180\n\t"
      "s_load_dword %7, %12, 0x1c0\n\t"
      "s_load_dword %8, %12, 0x200\n\t"
      "s_load_dword %9, %12, 0x240\n\t"
      "s_load_dword %10, %12, 0x280\n\t"
      "s_load_dword %11, %12, 0x2c0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(d0), "=&s"(d1), "=&s"(d2), "=&s"(d3), "=&s"(d4), "=&s"(d5), "=&s"(d6), "=&s"(d7), "=&s"(d8),
        "=&s"(d9), "=&s"(d10), "=&s"(d11)
      : "s"(k)
      : "memory");
}

// Grid exchange of a one-wave workgroup, in two halves.  cyc_arrive stores
// its statistics (feasible count, the taint / affinity raw maxima, lo) into
// its flag line as four words each tagged with `seq` in the high half (an
// aligned 8-byte store is single-copy atomic, so a word holding `seq` holds
// this call's value); cyc_await polls every line until all words hold `seq`
// (bounded; a timeout is sticky and reported) and folds them as it reads.
// Work issued between the two (the host rows) overlaps the wait.
// (Until round 5 the statistics went to a slot array read after the flags:
// one more dependent load round trip.)
__device__ __forceinline__ void cyc_arrive(const CycStatic& S, unsigned seq, const int32_t (&v)[4]) {
  const int lane = threadIdx.x;
  const uint32_t x = lane == 0 ? (uint32_t)v[0] : lane == 1 ? (uint32_t)v[1] : lane == 2 ? (uint32_t)v[2] : (uint32_t)v[3];
  if (lane < 4)
    gst(reinterpret_cast<unsigned long long*>(S.flags + (size_t)blockIdx.x * 32) + lane,
        ((unsigned long long)seq << 32) | x);
}

// v: [0] summed, [1..3] max (all non-negative), over every workgroup
__device__ __forceinline__ bool cyc_await(const CycStatic& S, unsigned seq, int G, int32_t (&v)[4]) {
  const int lane = threadIdx.x;
  unsigned spins = 0;
  for (;;) {
    bool ok = true;
    int32_t a = 0, b = 0, c = 0, d = 0;
    for (int l = lane; l < G; l += 64) {
      const unsigned long long* f = reinterpret_cast<const unsigned long long*>(S.flags + (size_t)l * 32);
      const unsigned long long w0 = gld(f), w1 = gld(f + 1), w2 = gld(f + 2), w3 = gld(f + 3);
      ok = ok && (unsigned)(w0 >> 32) == seq && (unsigned)(w1 >> 32) == seq && (unsigned)(w2 >> 32) == seq &&
           (unsigned)(w3 >> 32) == seq;
      a += (int32_t)(uint32_t)w0;
      b = max(b, (int32_t)(uint32_t)w1);
      c = max(c, (int32_t)(uint32_t)w2);
      d = max(d, (int32_t)(uint32_t)w3);
    }
    const bool done = __all(ok);
    bool give_up = false;
    if (!done) {
      __builtin_amdgcn_s_sleep(1);
      give_up = ++spins > (1u << 22) || gld(S.timeout);
      if (give_up && lane == 0) gst(S.timeout, 1u);
    }
    if (done || give_up) {
      v[0] = (int32_t)wreduce((uint32_t)a, OpAdd32{});
      v[1] = wreduce(b, OpMaxI32{});
      v[2] = wreduce(c, OpMaxI32{});
      v[3] = wreduce(d, OpMaxI32{});
      return done;
    }
  }
}

// A lane's nodes: indices, resource columns, the prefetched static columns.
// Every load unconditional and unmasked (clamped indices; a column past the
// allocated ones reads a valid word the evaluation never uses), so they are
// all in flight together; cyc_stage_nodes finishes them once they are in.
template <int KN>
__device__ __forceinline__ void cyc_load_nodes(const CycStatic& S, bool want_img, int G, int (&nk)[KN],
                                               NodeCols (&L)[KN], PNode (&nd)[KN], uint32_t (&lv)[KN][kCycLab],
                                               uint32_t (*s_lab)[kCycLab][64]) {
  const DevCluster& c = S.c;
  const int lane = threadIdx.x;
  const int N = c.N;
  const size_t NN = N;
  const int R = c.R, Lc = c.L, T = c.T, I = c.I;
  const uint32_t* tcol = T > 0 ? c.taints : (const uint32_t*)c.allowed;
  const uint32_t* icol = want_img && I > 0 ? c.images : (const uint32_t*)c.allowed;
  const int Tm = T > 0 ? T : 1, Im = want_img && I > 0 ? I : 1;
#pragma unroll
  for (int k = 0; k < KN; k++) {
    const int n = (k * G + (int)blockIdx.x) * 64 + lane;
    nk[k] = n;
    const int m = n < N ? n : N - 1;
#pragma unroll
    for (int r = 0; r < KSG_MAX_RES; r++) {
      const size_t o = (size_t)(r < R ? r : 0) * NN + m;
      L[k].alloc[r] = c.alloc[o];
      L[k].req[r] = S.requested[o];
    }
    L[k].nz_cpu = S.nonzero[m];
    L[k].nz_mem = S.nonzero[NN + m];
    L[k].pod_count = S.pod_count[m];
    L[k].allowed = c.allowed[m];
    nd[k].uns = c.unsched[m] != 0;
#pragma unroll
    for (int q = 0; q < kCycLab; q++) lv[k][q] = c.label_val[(size_t)(q < Lc ? q : 0) * NN + m];
#pragma unroll
    for (int q = 0; q < kCycTnt; q++) nd[k].tnt[q] = tcol[(size_t)(q < Tm ? q : 0) * NN + m];
#pragma unroll
    for (int q = 0; q < kCycImg; q++) nd[k].img[q] = icol[(size_t)(q < Im ? q : 0) * NN + m];
    nd[k].label_val = (const KSG_G1 uint32_t*)c.label_val;
    nd[k].label_num = (const KSG_G1 int64_t*)c.label_num;
    nd[k].label_num_ok = (const KSG_G1 uint8_t*)c.label_num_ok;
    nd[k].taints = (const KSG_G1 uint32_t*)c.taints;
    nd[k].taint_effect = (const KSG_G1 uint8_t*)c.taint_effect;
    nd[k].images = (const KSG_G1 uint32_t*)c.images;
    nd[k].N = NN;
    nd[k].n = m;
    nd[k].lab = (const KSG_L3 uint32_t*)&s_lab[k][0][lane];
  }
}

// The taint effects into LDS (issued behind the columns), then the masks and
// the label rows once the loads are in.
template <int KN>
__device__ __forceinline__ void cyc_stage_nodes(const CycStatic& S, NodeCols (&L)[KN], PNode (&nd)[KN],
                                                const uint32_t (&lv)[KN][kCycLab], uint32_t (*s_lab)[kCycLab][64],
                                                uint8_t* s_eff) {
  const DevCluster& c = S.c;
  const int lane = threadIdx.x;
  const int R = c.R, Lc = c.L;
  const bool eff_lds = c.V <= kCycEff;
  if (eff_lds)
    for (int i = lane; i < c.V; i += 64) s_eff[i] = c.taint_effect[i];
#pragma unroll
  for (int k = 0; k < KN; k++) {
#pragma unroll
    for (int r = 0; r < KSG_MAX_RES; r++) {
      L[k].alloc[r] = r < R ? L[k].alloc[r] : 0;
      L[k].req[r] = r < R ? L[k].req[r] : 0;
    }
#pragma unroll
    for (int q = 0; q < kCycLab; q++) s_lab[k][q][lane] = q < Lc ? lv[k][q] : 0;
    nd[k].eff_lds = eff_lds;
    nd[k].eff = (const KSG_L3 uint8_t*)s_eff;
  }
}

// One call on a wave whose nodes are loaded (L, nd) and whose pod programs are
// in LDS (P): the deferred assume, the staged append, the evaluation, the
// exchange, the rows.  K is the kernel arguments' copy (ksg_eval_cycle) or
// the LDS copy of the mailbox (ksg_cycle_server); podw its pod record as words.
template <int KN, bool SYS>
__device__ __forceinline__ void cyc_serve(const CycStatic& S, const CycCall& K, const int32_t* P,
                                          const int32_t* podw, const int (&nk)[KN], NodeCols (&L)[KN],
                                          const PNode (&nd)[KN], const uint32_t (&nsw)[KN], int G
#ifdef KSG_STAMPS
                                          , unsigned long long* y_acc, unsigned long long& y_last
#endif
) {
  const int lane = threadIdx.x;
  const DevCluster& c = S.c;
  const int N = c.N;
  const size_t NN = N;
  const ksg_pod& p = K.pod;
  if (K.wpods && blockIdx.x == 0) {   // the staged append: workgroup 0 copies it to the device pool
    constexpr int PW = (int)(sizeof(ksg_pod) / 4);
    if (lane < PW) reinterpret_cast<int32_t*>(K.wpods)[lane] = podw[lane];
    for (int64_t i = lane; i < K.slen; i += 64) K.wprog[i] = K.sprog[i];
  }
  // the deferred assume: NodeInfo.AddPod on the owner lane's node
#pragma unroll
  for (int k = 0; k < KN; k++)
    if (nk[k] == K.cm_node) {
      const int n = nk[k];
#pragma unroll
      for (int r = 0; r < KSG_MAX_RES; r++)
        if (r < c.R) {
          L[k].req[r] += K.cm_req[r];
          S.requested[(size_t)r * NN + n] = L[k].req[r];
        }
      L[k].nz_cpu += K.cm_nz_cpu;
      L[k].nz_mem += K.cm_nz_mem;
      L[k].pod_count += 1;
      S.nonzero[n] = L[k].nz_cpu;
      S.nonzero[NN + n] = L[k].nz_mem;
      S.pod_count[n] = L[k].pod_count;
    }
  KSG_YSTAMP(0);

  // ---- evaluate: every filter independently, then the first rejection in order ---------
  const int boff = p.blob;
  auto rb = [boff](int off) { return off < 0 ? -1 : off - boff; };
  const int32_t* tolf = P + rb(p.tol);
  const int32_t* tolp = tolf + c.W;
  const int na_req = rb(p.na_req), na_pref = rb(p.na_pref), img = rb(p.img), ports = rb(p.ports);
  const bool reject = (p.flags & KSG_POD_PREFILTER_REJECT) != 0;
  const bool has_nset = p.node_set >= 0;
  const CmProf cm{K.cm_fast != 0, K.cm_least != 0, K.cm_wc, K.cm_wm, K.cm_inv_ws, K.cm_inv_wc, K.cm_inv_wm};
  const uint32_t fm = K.fmask, sm = K.smask;
  uint32_t st[KN];
  int64_t part[KN], rt[KN], ra[KN], rf[KN], rbal[KN], rimg[KN];
#pragma unroll
  for (int k = 0; k < KN; k++) {
    const int n = nk[k];
    const PNode& x = nd[k];
    uint32_t w[KSG_NPLUGINS] = {};   // per-plugin status word (0: passes or not run)
    if (fm & bit(KSG_PL_NODE_UNSCHEDULABLE))
      w[KSG_PL_NODE_UNSCHEDULABLE] =
          (x.unsched() && !(p.flags & KSG_POD_TOL_UNSCHED)) ? KSG_PL_NODE_UNSCHEDULABLE + 1 : 0;
    if (fm & bit(KSG_PL_NODE_NAME))
      w[KSG_PL_NODE_NAME] = (p.node_name != -1 && p.node_name != n) ? KSG_PL_NODE_NAME + 1 : 0;
    int tslot;
    int64_t tscore;
    pnode_taints(x, c.T, tolf, tolp, (fm & bit(KSG_PL_TAINT_TOLERATION)) != 0,
                 (sm & bit(KSG_PL_TAINT_TOLERATION)) != 0, tslot, tscore);
    if (fm & bit(KSG_PL_TAINT_TOLERATION))
      w[KSG_PL_TAINT_TOLERATION] = tslot >= 0 ? (uint32_t)(KSG_PL_TAINT_TOLERATION + 1) | ((uint32_t)tslot << 8) : 0;
    if (fm & bit(KSG_PL_NODE_AFFINITY))
      w[KSG_PL_NODE_AFFINITY] =
          na_required_match(x, P, na_req) ? 0 : (uint32_t)(KSG_PL_NODE_AFFINITY + 1) | (1u << 8);
    if ((fm & bit(KSG_PL_NODE_PORTS)) && ports >= 0 && S.used_ports)
      w[KSG_PL_NODE_PORTS] =
          ports_conflict(S.used_ports, N, n < N ? n : N - 1, P + ports) ? KSG_PL_NODE_PORTS + 1 : 0;
    if (fm & bit(KSG_PL_NODE_RESOURCES_FIT)) {
      const uint32_t b = fit_filter(c, p, L[k], K.fit_ignored);
      w[KSG_PL_NODE_RESOURCES_FIT] = b ? (uint32_t)(KSG_PL_NODE_RESOURCES_FIT + 1) | (b << 8) : 0;
    }
    uint32_t s = 0;
    for (int kf = 0; kf < K.n_filter && !s; kf++) {
      const int pl = (int)((K.forder >> (4 * kf)) & 15u);
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < KSG_NPLUGINS; q++) v = pl == q ? w[q] : v;
      s = v;
    }
    if (reject || (has_nset && !((nsw[k] >> (n & 31)) & 1u))) s = KSG_FS_NOT_EVALUATED;
    st[k] = n < N ? s : (uint32_t)KSG_FS_NOT_EVALUATED;
    // raw scores of a feasible node
    part[k] = rt[k] = ra[k] = rf[k] = rbal[k] = rimg[k] = 0;
    if (st[k] == 0) {
      if (sm & (bit(KSG_PL_NODE_RESOURCES_FIT) | bit(KSG_PL_BALANCED_ALLOCATION))) {
        if (cm.fast) {
          fit_ba_cm(cm, p, L[k], rf[k], rbal[k]);
        } else {
          rf[k] = fit_score(*K.gprof, p, L[k]);
          rbal[k] = ba_score(*K.gprof, p, L[k]);
        }
        if (!(sm & bit(KSG_PL_NODE_RESOURCES_FIT))) rf[k] = 0;
        if (!(sm & bit(KSG_PL_BALANCED_ALLOCATION))) rbal[k] = 0;
      }
      if (sm & bit(KSG_PL_IMAGE_LOCALITY)) rimg[k] = pnode_image_score(x, c.I, P, img, p.n_containers);
      if (sm & bit(KSG_PL_TAINT_TOLERATION)) rt[k] = tscore;
      if (sm & bit(KSG_PL_NODE_AFFINITY)) ra[k] = na_pref_score(x, P, na_pref);
      part[k] = rf[k] * K.w_fit + rbal[k] * K.w_ba + rimg[k] * K.w_img;
    }
  }
  KSG_YSTAMP(1);

  // ---- this workgroup's statistics, the exchange ---------------------------------------
  int32_t feas = 0, mt = 0, ma = 0, lo = 0;
#pragma unroll
  for (int k = 0; k < KN; k++)
    if (st[k] == 0) {
      feas += 1;
      mt = max(mt, (int32_t)rt[k]);
      ma = max(ma, (int32_t)ra[k]);
      lo = max(lo, N - nk[k]);
    }
  {
    const int32_t mine[4] = {(int32_t)wreduce((uint32_t)feas, OpAdd32{}), wreduce(mt, OpMaxI32{}),
                             wreduce(ma, OpMaxI32{}), wreduce(lo, OpMaxI32{})};
    cyc_arrive(S, K.seq, mine);
  }
  const unsigned seq = K.seq;
  // ---- the rows that need no global fact, while the other workgroups arrive:
  // filter statuses and raw scores (as if Score runs; a call with fewer than
  // two feasible nodes, where it does not, zeroes its one feasible node's raw
  // values after the exchange)
  const int es = K.es;
#pragma unroll
  for (int k = 0; k < KN; k++) {
    const int n = nk[k];
    if (n >= N) continue;
    const bool ok = st[k] == 0;
    hst<SYS>(K.h_fs + n, st[k]);
    for (int q = 0; q < K.n_rows; q++) {
      const int pl = (int)((K.rows >> (4 * q)) & 15u);
      int64_t x = 0;
      if (ok && ((sm >> pl) & 1u))
        x = pl == KSG_PL_NODE_RESOURCES_FIT     ? rf[k]
            : pl == KSG_PL_BALANCED_ALLOCATION ? rbal[k]
            : pl == KSG_PL_IMAGE_LOCALITY      ? rimg[k]
            : pl == KSG_PL_TAINT_TOLERATION    ? rt[k]
            : pl == KSG_PL_NODE_AFFINITY       ? ra[k]
                                               : 0;
      cyc_put_es<SYS>(K.h_raw, (size_t)q * NN + n, x, es);
    }
  }
  KSG_YSTAMP(2);
  int32_t gs[4];
  const bool xok = cyc_await(S, seq, G, gs);
  KSG_YSTAMP(3);
  const int32_t nfeas = gs[0], max_t = gs[1], max_a = gs[2], low = gs[3];
  KSG_YSTAMP(4);

  // ---- selectHost over the normalised totals (not stored: the host derives the
  // normalised rows from the raw ones and the maxima, round 6) ---------------------------
  const bool scored = nfeas >= 2;   // fewer than two feasible nodes: no Score ran, nothing recorded
  PodView v{};                       // total_score's inputs
  v.smask = sm;
  v.w_t = K.w_t;
  v.w_a = K.w_a;
  uint64_t key = 0;
  uint32_t err = 0;
#pragma unroll
  for (int k = 0; k < KN; k++) {
    const int n = nk[k];
    if (n >= N) continue;
    const bool ok = st[k] == 0;
    if (scored && ok) {
      const int64_t total = total_score(v, part[k], rt[k], ra[k], max_t, max_a, err, nullptr, nullptr);
      const uint64_t kk = argmax_key(total, n);
      key = kk > key ? kk : key;
    }
    if (!scored && ok)   // no Score ran: nothing recorded for it
      for (int q = 0; q < K.n_rows; q++) cyc_put_es<SYS>(K.h_raw, (size_t)q * NN + n, 0, es);
  }
  key = wreduce(key, OpMaxU64{});
  err = wreduce(err, OpOr32{});
  // Completion: one word for the host.  Every workgroup folds its selectHost
  // key and error bits into this call's slot with agent-scope atomics, waits
  // for its host rows (system-scope stores: vmcnt(0) means performed), and
  // arrives on a counter; the last to arrive reads the slots and stores the
  // result line (statistics, best key, error bits) and then its done word,
  // taking the slots' values with exchanges that leave them zero for the next
  // call (which starts only after the host has seen this one's done word, so
  // the sequence numbers need not be consecutive).
  // (Round 4: one record per workgroup, which the host polled one by one.)
  unsigned long long* kslot = S.key;
  if (lane == 0) {
    __hip_atomic_fetch_max((__attribute__((address_space(1))) unsigned long long*)kslot, (unsigned long long)key,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (err | (xok ? 0u : 2u))
      __hip_atomic_fetch_or((__attribute__((address_space(1))) unsigned*)(S.errw), err | (xok ? 0u : 2u),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  host_release<SYS>();   // this wave's rows and atomics are performed
  KSG_YSTAMP(5);
  if (lane == 0) {
    const unsigned old = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)S.arrive, 1u,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1) % (unsigned)G == 0) {   // the last workgroup of this call
      const unsigned long long best = __hip_atomic_exchange(
          (__attribute__((address_space(1))) unsigned long long*)kslot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned e = __hip_atomic_exchange((__attribute__((address_space(1))) unsigned*)S.errw, 0u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int32_t* h = K.h_stats;
      hst<SYS>(h + 0, nfeas);
      hst<SYS>(h + 1, max_t);
      hst<SYS>(h + 2, max_a);
      hst<SYS>(h + 3, low);
      hst<SYS>(reinterpret_cast<unsigned long long*>(h + 4), best);
      hst<SYS>(reinterpret_cast<uint32_t*>(h + 6), e);
      host_release<SYS>();
      __hip_atomic_store(reinterpret_cast<unsigned*>(h + 7), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  KSG_YSTAMP(6);
}

#ifdef KSG_STAMPS
#define KSG_YSTAMP_ARGS , y_acc, y_last
#else
#define KSG_YSTAMP_ARGS
#endif

template <int KN, bool SYS>
__global__ __launch_bounds__(64) void ksg_eval_cycle(CycArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ uint8_t s_eff[kCycEff];
  __shared__ uint32_t s_lab[KN][kCycLab][64];
  const int lane = threadIdx.x;
  const int G = (int)gridDim.x;
#ifdef KSG_STAMPS
  unsigned long long y_acc[8] = {}, y_last = __builtin_amdgcn_s_memtime();
#endif
  // ---- entry: argument lines, node columns, programs, all in flight together ----------
  static_assert(offsetof(CycArgs, blob) <= 768 && sizeof(CycArgs) >= 768, "cyc_warm_args covers 12 lines");
  cyc_warm_args();
  const CycStatic& S = a.s;
  const CycCall& K = a.k;
  const int N = S.c.N;
  const int blen = K.blob_len;
  int nk[KN];
  NodeCols L[KN];
  PNode nd[KN];
  uint32_t lv[KN][kCycLab];
  uint32_t nsw[KN];
  cyc_load_nodes<KN>(S, (K.smask >> KSG_PL_IMAGE_LOCALITY) & 1u, G, nk, L, nd, lv, s_lab);
  const int32_t* nsrc = K.pod.node_set >= 0 ? K.gprog + K.pod.node_set : S.c.allowed;
#pragma unroll
  for (int k = 0; k < KN; k++) nsw[k] = (uint32_t)nsrc[(nk[k] < N ? nk[k] : N - 1) >> 5];
  // the pod's programs into LDS (issued behind the columns)
  const __attribute__((address_space(4))) char* kbase =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  if (blen <= kCycBlob) {
    const __attribute__((address_space(4))) int32_t* kb =
        (const __attribute__((address_space(4))) int32_t*)(kbase + offsetof(CycArgs, blob));
    int32_t w[kCycBlob / 64];
#pragma unroll
    for (int u = 0; u < kCycBlob / 64; u++) w[u] = kb[lane + 64 * u];   // inside the arguments: unconditional
#pragma unroll
    for (int u = 0; u < kCycBlob / 64; u++)
      if (lane + 64 * u < blen) s_blob[lane + 64 * u] = w[u];
  } else {
    for (int i = lane; i < blen; i += 64) s_blob[i] = K.bsrc[i];
  }
  cyc_stage_nodes<KN>(S, L, nd, lv, s_lab, s_eff);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS copies visible to the (single) wave
  const int32_t* podw =
      (const int32_t*)(const __attribute__((address_space(4))) int32_t*)(kbase + offsetof(CycArgs, k) +
                                                                         offsetof(CycCall, pod));
  cyc_serve<KN, SYS>(S, K, s_blob, podw, nk, L, nd, nsw, G KSG_YSTAMP_ARGS);
#ifdef KSG_STAMPS
  if (lane == 0 && blockIdx.x == 0 && S.stamps)
    for (int i = 0; i < 7; i++) atomicAdd(&S.stamps[i], y_acc[i]);
#endif
}

// System-scope load of host memory (the mailbox): around the GPU caches.
template <class T>
__device__ __forceinline__ T sys_ld(const T* p) {
  return __hip_atomic_load((__attribute__((address_space(1))) T*)(const_cast<T*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// The persistent form.  With the mailbox in fine-grained device memory
// (SrvArgs::direct, the default where the CPU maps it: round 6) every
// workgroup polls its sequence word and reads the call in place: HBM, not
// PCIe, so no relay.  Otherwise (pinned host memory):
// workgroup 0 alone polls the host mailbox (lane 0,
// one PCIe read in flight at a time), reads the call and its programs, and
// relays them into device memory behind a go word (agent-scope stores); the
// other workgroups poll the go word and read the relayed copy, so PCIe carries
// one poll and one call per cycle (every workgroup polling the host line
// measured 59 us per call: the host side of the cycle slowed down too).  A
// workgroup leaves on op = 1 (stop), after kSrvIdle without a new call, or when
// an exchange timed out (the host then finds the launch finished without its
// done words and fails loudly).  Node columns stay in registers / LDS: only
// this kernel changes them while it runs (the deferred assumes, written back).
template <int KN, bool SYS>
__global__ __launch_bounds__(64) void ksg_cycle_server(SrvArgs a) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ uint8_t s_eff[kCycEff];
  __shared__ uint32_t s_lab[KN][kCycLab][64];
  __shared__ __attribute__((aligned(16))) CycCall s_k;
  const int lane = threadIdx.x;
  const int G = (int)gridDim.x;
  const CycStatic& S = a.s;
  const int N = S.c.N;
  const bool direct = a.direct != 0;
  const bool relay = !direct && blockIdx.x == 0;
  int nk[KN];
  NodeCols L[KN];
  PNode nd[KN];
  uint32_t lv[KN][kCycLab];
  uint32_t nsw[KN];
  cyc_load_nodes<KN>(S, a.want_img != 0, G, nk, L, nd, lv, s_lab);
  cyc_stage_nodes<KN>(S, L, nd, lv, s_lab, s_eff);
  const SrvMailbox* mb = a.mb;
  unsigned last = a.last;
#ifdef KSG_STAMPS
  unsigned long long y_acc[8] = {}, y_last = __builtin_amdgcn_s_memtime();
#endif
  constexpr int KW = (int)(sizeof(CycCall) / 4);
  for (;;) {
    // ---- wait for the next call: the host line (workgroup 0) or the go word -------------
    unsigned seq = last;
    if (lane == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        seq = relay || direct ? sys_ld(&mb->seq) : gld(a.d_go);
        if (seq != last) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSrvIdle || gld(S.timeout)) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    seq = (unsigned)__builtin_amdgcn_readfirstlane((int)seq);
    if (seq == last) break;   // idle or a timed-out exchange elsewhere: leave
    // ---- the call and its programs into LDS (workgroup 0: from the host, relayed) -------
    if (direct) {   // the mailbox in device memory: read it in place (system scope: the CPU wrote it)
      // the call and the first kCycBlob program words in one round trip (the
      // words past the call's blob_len are read and dropped)
      const int32_t* src = reinterpret_cast<const int32_t*>(&mb->k);
      int32_t bw[kCycBlob / 64];
#pragma unroll
      for (int u = 0; u < kCycBlob / 64; u++) bw[u] = sys_ld(mb->blob + lane + 64 * u);
      for (int i = lane; i < KW; i += 64) reinterpret_cast<int32_t*>(&s_k)[i] = sys_ld(src + i);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const int blen = s_k.op != 0 ? 0 : s_k.blob_len;
#pragma unroll
      for (int u = 0; u < kCycBlob / 64; u++)
        if (lane + 64 * u < blen) s_blob[lane + 64 * u] = bw[u];
      for (int i = kCycBlob + lane; i < blen; i += 64) s_blob[i] = sys_ld(mb->blob + i);
    } else if (relay) {
      const int32_t* src = reinterpret_cast<const int32_t*>(&mb->k);
      int32_t* dst = reinterpret_cast<int32_t*>(a.d_call);
      for (int i = lane; i < KW; i += 64) {
        const int32_t x = sys_ld(src + i);
        reinterpret_cast<int32_t*>(&s_k)[i] = x;
        gst(dst + i, x);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const int blen = s_k.op != 0 ? 0 : s_k.blob_len;
      for (int i = lane; i < blen; i += 64) {
        const int32_t x = sys_ld(mb->blob + i);
        s_blob[i] = x;
        gst(a.d_blob + i, x);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the relayed words are stored ...
      if (lane == 0) gst(a.d_go, seq);                     // ... before the go word
    } else {
      const int32_t* src = reinterpret_cast<const int32_t*>(a.d_call);
      for (int i = lane; i < KW; i += 64) reinterpret_cast<int32_t*>(&s_k)[i] = gld(src + i);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const int blen = s_k.op != 0 ? 0 : s_k.blob_len;
      for (int i = lane; i < blen; i += 64) s_blob[i] = gld(a.d_blob + i);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (s_k.op != 0) break;   // stop
    if (s_k.pod.node_set >= 0) {   // the PreFilterResult's node bitmap (one more round trip, only then)
      const int32_t* nsrc = s_k.gprog + s_k.pod.node_set;
#pragma unroll
      for (int k = 0; k < KN; k++) nsw[k] = (uint32_t)nsrc[(nk[k] < N ? nk[k] : N - 1) >> 5];
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
#pragma unroll
      for (int k = 0; k < KN; k++) nsw[k] = 0xffffffffu;
    }
#ifdef KSG_STAMPS
    y_last = __builtin_amdgcn_s_memtime();
#endif
    cyc_serve<KN, SYS>(S, s_k, s_blob, reinterpret_cast<const int32_t*>(&s_k.pod), nk, L, nd, nsw,
                       G KSG_YSTAMP_ARGS);
    last = seq;
    if (gld(S.timeout)) break;   // an exchange gave up: every workgroup leaves
  }
#ifdef KSG_STAMPS
  if (lane == 0 && blockIdx.x == 0 && S.stamps)
    for (int i = 0; i < 7; i++) atomicAdd(&S.stamps[i], y_acc[i]);
#endif
}
