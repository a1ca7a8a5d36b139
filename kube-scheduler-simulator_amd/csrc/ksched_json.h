// Device serialiser of the result-store annotations (SURVEY.md §8(f) rank 1;
// VERDICT r4 item 5): the filter-result, score-result and finalscore-result
// values of every pod of a captured queue run, written on the device from the
// capture rows still in HBM, byte-identical to ksg_annotate
// (ksched_annotate.cpp, itself Go encoding/json of store.go:423-507's maps).
// The host receives finished bytes instead of capture rows plus a CPU pass.
//
// Three kernels per chunk of pods:
//   ksg_json_len    S workgroups per pod (node segments in name order), lanes
//                   over contiguous runs of a segment: the segment's byte
//                   counts and emitted entries per value;
//   ksg_json_scan   one workgroup: segment prefixes, value lengths, and the
//                   byte offset of every value (pod-major);
//   ksg_json_write  S workgroups per pod again, rounds of kJsonWBlock
//                   consecutive nodes (one per lane): a workgroup scan of the
//                   entries' lengths places each entry in an LDS window, and
//                   the window goes out as lane-consecutive (coalesced) byte
//                   stores.  A lane writing its own run straight to HBM made
//                   every store instruction touch 64 lines (3.7 ms per
//                   64-pod chunk at 15,000 nodes) and slowed the concurrent
//                   copy back of the previous chunk.
// Every string piece (quoted node keys, plugin keys, messages) arrives
// escaped from the host annotator; the device only copies pieces and formats
// integers.
#pragma once

namespace ksk {

constexpr int kJsonBlock = 256;
constexpr int kJsonWBlock = 128;        // ksg_json_write: nodes per round
constexpr int kJsonWin = 40 * 1024;     // ksg_json_write: LDS window bytes

struct JsonTables {
  const char* node_keys;          // node n's "<name>": at node_key_off[n]
  const int64_t* node_key_off;    // [N + 1]
  const int32_t* node_order;      // [N] node indices sorted bytewise by name
  const char* plugin_keys;        // plugin p's "<name>": at plugin_key_off[p]
  const int32_t* plugin_key_off;  // [KSG_NPLUGINS + 1]
  int32_t by_name[KSG_NPLUGINS];  // plugin ids sorted by name
  const char* msgs;               // quoted, escaped static messages: index pl * 8 + reason
  const int32_t* msg_off;         // [KSG_NPLUGINS * 8 + 1]; an empty slot has length 0
  const char* taint_msgs;         // "node(s) had untolerated taint {k: v}" per taint-vocab id, quoted
  const int32_t* taint_msg_off;   // [V + 1]
  const char* fit_parts;          // escaped, unquoted: "Too many pods", then "Insufficient <res r>"
  const int32_t* fit_part_off;    // [1 + R + 1]
  int32_t n_res;
  int32_t n_taint_vocab;
};

struct JsonArgs {
  JsonTables t;
  int32_t N;
  int32_t T;                      // taint slots per node
  const uint32_t* taints;         // [T][N]
  const ksg_pod* pods;            // the context's pod records (filter_skip)
  int32_t first;                  // queue index of pod 0 of the chunk
  const ksg_result* res;          // [count]
  const uint32_t* fstatus;        // [count][N]
  const int64_t* raw;             // [count][n_rows][N]
  const int64_t* norm;            // [count][n_rows][N]
  int32_t n_rows;
  int32_t row_of[KSG_NPLUGINS];   // capture row of plugin p, -1 none
  int32_t n_filter;
  int32_t filter_order[KSG_NPLUGINS];
  uint32_t score_mask;
  uint32_t normalize_mask;
  int64_t weight[KSG_NPLUGINS];   // the Store's score weights
  int32_t count;                  // pods in the chunk
  int32_t S;                      // node segments per pod (workgroups per pod)
  int64_t* segtot;                // [count][S][5] per-segment counts
  int64_t* segoff;                // [count][S][6] bytes / entries before the segment, per value
  int64_t* totals;                // [count * 3] bytes of each value
  int64_t* offsets;               // [count * 3 + 1] (ksg_json_scan)
  char* out;                      // the values back to back
  uint32_t* err;                  // a status word without a message
};

// The pod's plugin sets: filter plugins that ran (run positions), score
// plugins that ran, as ksg_annotate's caller (bulk.py BulkAnnotator._order)
// derives them from filter_skip, the IPA PreFilter bit and score_skip.
struct JsonPod {
  int8_t pos[KSG_NPLUGINS];       // run position of a filter plugin that ran, -1 otherwise
  uint32_t fset;                  // filter plugins that ran
  uint32_t sset;                  // score plugins that ran (n_feasible >= 2)
  int32_t nf;
  int32_t pass_len;               // a passing node's body: {"A":"passed",...}
};

__device__ __forceinline__ JsonPod json_pod(const JsonArgs& a, int k) {
  JsonPod q;
  const ksg_pod& p = a.pods[a.first + k];
  const ksg_result r = a.res[k];
  uint32_t fskip = p.filter_skip;
  if (r.status & KSG_ST_IPA_PREFILTER_SKIP) fskip |= 1u << KSG_PL_INTER_POD_AFFINITY;
  for (int i = 0; i < KSG_NPLUGINS; i++) q.pos[i] = -1;
  q.fset = 0;
  int np = 0;
  for (int i = 0; i < a.n_filter; i++) {
    const int pl = a.filter_order[i];
    if ((fskip >> pl) & 1u) continue;
    q.pos[pl] = (int8_t)np++;
    q.fset |= 1u << pl;
  }
  q.nf = r.n_feasible;
  q.sset = r.n_feasible >= 2 ? (a.score_mask & ~r.score_skip) : 0u;
  int len = 2;
  int cnt = 0;
  for (int i = 0; i < KSG_NPLUGINS; i++) {
    const int pl = a.t.by_name[i];
    if (!((q.fset >> pl) & 1u)) continue;
    len += (a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl]) + 8 + (cnt ? 1 : 0);
    cnt++;
  }
  q.pass_len = len;
  return q;
}

__device__ __forceinline__ int dec_len(uint64_t u) {
  int d = 1;
  while (u >= 10) { u /= 10; d++; }
  return d;
}

// "<v>" (quoted decimal) length
__device__ __forceinline__ int qint_len(int64_t v) {
  const uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  return 2 + dec_len(u) + (v < 0 ? 1 : 0);
}

__device__ __forceinline__ char* put_qint(char* o, int64_t v) {
  const uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  const int d = dec_len(u);
  *o++ = '"';
  if (v < 0) *o++ = '-';
  uint64_t x = u;
  for (int i = d - 1; i >= 0; i--) {
    o[i] = (char)('0' + x % 10);
    x /= 10;
  }
  o += d;
  *o++ = '"';
  return o;
}

__device__ __forceinline__ char* put_bytes(char* o, const char* s, int64_t n) {
  for (int64_t i = 0; i < n; i++) o[i] = s[i];
  return o + n;
}

// The rejecting plugin's message (quoted JSON) for status word st at node n:
// its length, and (o != nullptr) its bytes.  -1: no message for this word.
__device__ __forceinline__ int msg_piece(const JsonArgs& a, uint32_t st, int n, char* o) {
  const int pl = (int)(st & 0xFF) - 1;
  const uint32_t reason = st >> 8;
  const JsonTables& t = a.t;
  if (pl == KSG_PL_TAINT_TOLERATION) {
    if ((int)reason >= a.T) return -1;
    const uint32_t id = a.taints[(size_t)reason * a.N + n];
    if (id == 0 || (int)id > t.n_taint_vocab) return -1;
    const int b = t.taint_msg_off[id - 1], e = t.taint_msg_off[id];
    if (o) put_bytes(o, t.taint_msgs + b, e - b);
    return e - b;
  }
  if (pl == KSG_PL_NODE_RESOURCES_FIT) {   // fitsRequest order: pods, then columns
    int len = 2;
    bool first = true;
    char* w = o;
    if (w) *w++ = '"';
    for (int r = -1; r < t.n_res; r++) {
      if (!((reason >> (r + 1)) & 1u)) continue;
      const int b = t.fit_part_off[r + 1], e = t.fit_part_off[r + 2];
      len += (e - b) + (first ? 0 : 2);
      if (w) {
        if (!first) { *w++ = ','; *w++ = ' '; }
        w = put_bytes(w, t.fit_parts + b, e - b);
      }
      first = false;
    }
    if (w) *w++ = '"';
    return len;
  }
  if (pl < 0 || pl >= KSG_NPLUGINS || reason >= 8) return -1;
  const int b = t.msg_off[pl * 8 + reason], e = t.msg_off[pl * 8 + reason + 1];
  if (e == b) return -1;
  if (o) put_bytes(o, t.msgs + b, e - b);
  return e - b;
}

// One node's filter body ({...} after its key): length, and bytes when o.
__device__ __forceinline__ int filter_body(const JsonArgs& a, const JsonPod& q, uint32_t st, int n, char* o,
                                           uint32_t& err) {
  if (st == 0) {
    if (o) {
      *o++ = '{';
      bool first = true;
      for (int i = 0; i < KSG_NPLUGINS; i++) {
        const int pl = a.t.by_name[i];
        if (!((q.fset >> pl) & 1u)) continue;
        if (!first) *o++ = ',';
        first = false;
        o = put_bytes(o, a.t.plugin_keys + a.t.plugin_key_off[pl], a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl]);
        o = put_bytes(o, "\"passed\"", 8);
      }
      *o++ = '}';
    }
    return q.pass_len;
  }
  const int fail = (int)(st & 0xFF) - 1;
  const int last = fail >= 0 && fail < KSG_NPLUGINS ? q.pos[fail] : -1;
  if (last < 0) {   // rejected by a plugin that did not run
    err |= 1u;
    return 2;
  }
  int len = 2;
  bool first = true;
  if (o) *o++ = '{';
  for (int i = 0; i < KSG_NPLUGINS; i++) {
    const int pl = a.t.by_name[i];
    if (!((q.fset >> pl) & 1u) || q.pos[pl] > last) continue;
    const int kl = a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl];
    if (!first) {
      len += 1;
      if (o) *o++ = ',';
    }
    first = false;
    len += kl;
    if (o) o = put_bytes(o, a.t.plugin_keys + a.t.plugin_key_off[pl], kl);
    if (pl == fail) {
      const int ml = msg_piece(a, st, n, o);
      if (ml < 0) {
        err |= 2u;
        return len;
      }
      len += ml;
      if (o) o += ml;
    } else {
      len += 8;
      if (o) o = put_bytes(o, "\"passed\"", 8);
    }
  }
  if (o) *o++ = '}';
  return len;
}

// One feasible node's score (fin = false) or finalscore body.
__device__ __forceinline__ int score_body(const JsonArgs& a, const JsonPod& q, int k, int n, bool fin, char* o) {
  int len = 2;
  bool first = true;
  if (o) *o++ = '{';
  const size_t NN = a.N;
  for (int i = 0; i < KSG_NPLUGINS; i++) {
    const int pl = a.t.by_name[i];
    if (!((q.sset >> pl) & 1u)) continue;
    const int kl = a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl];
    if (!first) {
      len += 1;
      if (o) *o++ = ',';
    }
    first = false;
    len += kl;
    if (o) o = put_bytes(o, a.t.plugin_keys + a.t.plugin_key_off[pl], kl);
    const int row = a.row_of[pl];
    int64_t raw = 0, v;
    if (row >= 0) raw = a.raw[((size_t)k * a.n_rows + row) * NN + n];
    if (!fin) {
      v = raw;
    } else {
      const int64_t f = ((a.normalize_mask >> pl) & 1u) && row >= 0 ? a.norm[((size_t)k * a.n_rows + row) * NN + n] : raw;
      v = (int64_t)((uint64_t)f * (uint64_t)a.weight[pl]);   // Go int64 multiplication wraps
    }
    len += qint_len(v);
    if (o) o = put_qint(o, v);
  }
  if (first) {   // no score plugin: "{}"
    if (o) *o++ = '}';
    return len;
  }
  if (o) *o++ = '}';
  return len;
}

// Workgroup-exclusive scan of one int64 per lane (kJsonBlock lanes).
__device__ __forceinline__ int64_t block_exscan(int64_t x, int64_t* s_buf, int64_t& total) {
  const int tid = threadIdx.x;
  s_buf[tid] = x;
  __syncthreads();
  for (int d = 1; d < kJsonBlock; d <<= 1) {
    const int64_t y = tid >= d ? s_buf[tid - d] : 0;
    __syncthreads();
    s_buf[tid] += y;
    __syncthreads();
  }
  total = s_buf[kJsonBlock - 1];
  const int64_t incl = s_buf[tid];
  __syncthreads();
  return incl - x;
}

// The nodes (name order) of segment `seg` of a pod, split over the lanes.
__device__ __forceinline__ void lane_range(const JsonArgs& a, int seg, int tid, int& k0, int& k1) {
  const int N = a.N;
  const int per_seg = (N + a.S - 1) / a.S;
  const int s0 = min(N, seg * per_seg), s1 = min(N, s0 + per_seg);
  const int per = (s1 - s0 + kJsonBlock - 1) / kJsonBlock;
  k0 = min(s1, s0 + tid * per);
  k1 = min(s1, k0 + per);
}

// grid: count * S workgroups; workgroup (pod k, segment seg)
__global__ __launch_bounds__(kJsonBlock) void ksg_json_len(JsonArgs a) {
  __shared__ JsonPod s_q;
  __shared__ int64_t s_buf[kJsonBlock];
  const int k = blockIdx.x / a.S, seg = blockIdx.x % a.S, tid = threadIdx.x;
  if (tid == 0) s_q = json_pod(a, k);
  __syncthreads();
  const JsonPod& q = s_q;   // read in LDS: pos[] is indexed by plugin (a private copy would live in scratch)
  const int N = a.N;
  int k0, k1;
  lane_range(a, seg, tid, k0, k1);
  int64_t lf = 0, cf = 0, ls = 0, lt = 0, cs = 0;
  uint32_t err = 0;
  const bool scored = q.nf >= 2 && q.sset != 0;
  for (int j = k0; j < k1; j++) {
    const int n = a.t.node_order[j];
    const uint32_t st = a.fstatus[(size_t)k * N + n];
    if (st == KSG_FS_NOT_EVALUATED) continue;
    const int64_t kl = a.t.node_key_off[n + 1] - a.t.node_key_off[n];
    if (q.fset) {
      lf += kl + filter_body(a, q, st, n, nullptr, err);
      cf += 1;
    }
    if (scored && st == 0) {
      ls += kl + score_body(a, q, k, n, false, nullptr);
      lt += kl + score_body(a, q, k, n, true, nullptr);
      cs += 1;
    }
  }
  if (err) atomicOr(a.err, err);
  int64_t t[5];
  (void)block_exscan(lf, s_buf, t[0]);
  (void)block_exscan(cf, s_buf, t[1]);
  (void)block_exscan(ls, s_buf, t[2]);
  (void)block_exscan(lt, s_buf, t[3]);
  (void)block_exscan(cs, s_buf, t[4]);
  if (tid == 0)
    for (int i = 0; i < 5; i++) a.segtot[(size_t)blockIdx.x * 5 + i] = t[i];
}

// One workgroup: per pod (one lane each) the segments' prefixes and the
// three values' lengths (braces, a comma between entries); then the byte
// offset of every value, pod-major.
__global__ __launch_bounds__(kJsonBlock) void ksg_json_scan(JsonArgs a) {
  __shared__ int64_t s_buf[kJsonBlock];
  const int S = a.S;
  for (int k = threadIdx.x; k < a.count; k += kJsonBlock) {
    int64_t bf = 0, nf = 0, bs = 0, bt = 0, ns = 0;
    for (int g = 0; g < S; g++) {
      const int64_t* t = a.segtot + ((size_t)k * S + g) * 5;
      int64_t* o = a.segoff + ((size_t)k * S + g) * 6;
      o[0] = bf; o[1] = nf; o[2] = bs; o[3] = ns; o[4] = bt; o[5] = ns;
      bf += t[0]; nf += t[1]; bs += t[2]; bt += t[3]; ns += t[4];
    }
    a.totals[3 * k + 0] = 2 + bf + (nf > 0 ? nf - 1 : 0);
    a.totals[3 * k + 1] = 2 + bs + (ns > 0 ? ns - 1 : 0);
    a.totals[3 * k + 2] = 2 + bt + (ns > 0 ? ns - 1 : 0);
  }
  __syncthreads();
  const int n = 3 * a.count;
  int64_t carry = 0;
  for (int b = 0; b < n; b += kJsonBlock) {
    const int i = b + (int)threadIdx.x;
    const int64_t x = i < n ? a.totals[i] : 0;
    int64_t tot;
    const int64_t ex = block_exscan(x, s_buf, tot);
    if (i < n) a.offsets[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) a.offsets[n] = carry;
}

// Bytes of one entry into an LDS window [lo, hi) of the value: pos is the
// entry's position in the value; bytes outside the window are dropped (a
// later window pass writes them).
struct JsonWin {
  char* buf;
  int64_t lo, hi, pos;
  __device__ __forceinline__ void c(char ch) {
    if (pos >= lo && pos < hi) buf[pos - lo] = ch;
    pos++;
  }
  __device__ __forceinline__ void s(const char* p, int64_t n) {
    for (int64_t i = 0; i < n; i++) c(p[i]);
  }
  __device__ __forceinline__ void qint(int64_t v) {
    const uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    const int d = dec_len(u);
    c('"');
    if (v < 0) c('-');
    uint64_t x = u;
    for (int i = d - 1; i >= 0; i--) {   // digits in place, last first
      const int64_t at = pos + i;
      if (at >= lo && at < hi) buf[at - lo] = (char)('0' + x % 10);
      x /= 10;
    }
    pos += d;
    c('"');
  }
};

// msg_piece's bytes (its length was checked by ksg_json_len)
__device__ __forceinline__ void emit_msg(JsonWin& w, const JsonArgs& a, uint32_t st, int n) {
  const int pl = (int)(st & 0xFF) - 1;
  const uint32_t reason = st >> 8;
  const JsonTables& t = a.t;
  if (pl == KSG_PL_TAINT_TOLERATION) {
    if ((int)reason >= a.T) return;
    const uint32_t id = a.taints[(size_t)reason * a.N + n];
    if (id == 0 || (int)id > t.n_taint_vocab) return;
    w.s(t.taint_msgs + t.taint_msg_off[id - 1], t.taint_msg_off[id] - t.taint_msg_off[id - 1]);
    return;
  }
  if (pl == KSG_PL_NODE_RESOURCES_FIT) {   // fitsRequest order: pods, then columns
    bool first = true;
    w.c('"');
    for (int r = -1; r < t.n_res; r++) {
      if (!((reason >> (r + 1)) & 1u)) continue;
      if (!first) {
        w.c(',');
        w.c(' ');
      }
      w.s(t.fit_parts + t.fit_part_off[r + 1], t.fit_part_off[r + 2] - t.fit_part_off[r + 1]);
      first = false;
    }
    w.c('"');
    return;
  }
  if (pl < 0 || pl >= KSG_NPLUGINS || reason >= 8) return;
  w.s(t.msgs + t.msg_off[pl * 8 + reason], t.msg_off[pl * 8 + reason + 1] - t.msg_off[pl * 8 + reason]);
}

// filter_body's bytes
__device__ __forceinline__ void emit_filter(JsonWin& w, const JsonArgs& a, const JsonPod& q, uint32_t st, int n) {
  const int fail = st == 0 ? -2 : (int)(st & 0xFF) - 1;
  const int last = st == 0 ? KSG_NPLUGINS : (fail >= 0 && fail < KSG_NPLUGINS ? q.pos[fail] : -1);
  w.c('{');
  if (last < 0) {   // rejected by a plugin that did not run (ksg_json_len flagged it)
    w.c('}');
    return;
  }
  bool first = true;
  for (int i = 0; i < KSG_NPLUGINS; i++) {
    const int pl = a.t.by_name[i];
    if (!((q.fset >> pl) & 1u) || q.pos[pl] > last) continue;
    if (!first) w.c(',');
    first = false;
    w.s(a.t.plugin_keys + a.t.plugin_key_off[pl], a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl]);
    if (pl == fail) {
      emit_msg(w, a, st, n);
    } else {
      w.s("\"passed\"", 8);
    }
  }
  w.c('}');
}

// score_body's bytes
__device__ __forceinline__ void emit_score(JsonWin& w, const JsonArgs& a, const JsonPod& q, int k, int n, bool fin) {
  const size_t NN = a.N;
  bool first = true;
  w.c('{');
  for (int i = 0; i < KSG_NPLUGINS; i++) {
    const int pl = a.t.by_name[i];
    if (!((q.sset >> pl) & 1u)) continue;
    if (!first) w.c(',');
    first = false;
    w.s(a.t.plugin_keys + a.t.plugin_key_off[pl], a.t.plugin_key_off[pl + 1] - a.t.plugin_key_off[pl]);
    const int row = a.row_of[pl];
    int64_t raw = 0, v;
    if (row >= 0) raw = a.raw[((size_t)k * a.n_rows + row) * NN + n];
    if (!fin) {
      v = raw;
    } else {
      const int64_t f = ((a.normalize_mask >> pl) & 1u) && row >= 0 ? a.norm[((size_t)k * a.n_rows + row) * NN + n] : raw;
      v = (int64_t)((uint64_t)f * (uint64_t)a.weight[pl]);   // Go int64 multiplication wraps
    }
    w.qint(v);
  }
  w.c('}');
}

// Workgroup-exclusive scan of one int64 per lane (kJsonWBlock lanes).
__device__ __forceinline__ int64_t wblock_exscan(int64_t x, int64_t* s_buf, int64_t& total) {
  const int tid = threadIdx.x;
  s_buf[tid] = x;
  __syncthreads();
  for (int d = 1; d < kJsonWBlock; d <<= 1) {
    const int64_t y = tid >= d ? s_buf[tid - d] : 0;
    __syncthreads();
    s_buf[tid] += y;
    __syncthreads();
  }
  total = s_buf[kJsonWBlock - 1];
  const int64_t incl = s_buf[tid];
  __syncthreads();
  return incl - x;
}

// grid: count * S workgroups of kJsonWBlock lanes; workgroup (pod k, segment
// seg).  A value is '{' + entries joined by ',' + '}': entry g (g > 0) is
// written with its leading comma, so the value's first and last bytes (seg
// 0's lane 0) are never touched by another workgroup.
__global__ __launch_bounds__(kJsonWBlock) void ksg_json_write(JsonArgs a) {
  __shared__ JsonPod s_q;
  __shared__ int64_t s_buf[kJsonWBlock];
  __shared__ char s_win[kJsonWin];
  const int k = blockIdx.x / a.S, seg = blockIdx.x % a.S, tid = threadIdx.x;
  if (tid == 0) s_q = json_pod(a, k);
  __syncthreads();
  const JsonPod& q = s_q;   // read in LDS: pos[] is indexed by plugin (a private copy would live in scratch)
  const int N = a.N;
  const int per_seg = (N + a.S - 1) / a.S;
  const int s0 = min(N, seg * per_seg), s1 = min(N, s0 + per_seg);
  const int64_t* so = a.segoff + (size_t)blockIdx.x * 6;
  const bool scored = q.nf >= 2 && q.sset != 0;
  constexpr int64_t kLow = ((int64_t)1 << 40) - 1;
  for (int v = 0; v < 3; v++) {
    if (v == 0 ? !q.fset : !scored) continue;   // "{}" (seg 0's braces below)
    char* const out = a.out + a.offsets[3 * k + v];
    int64_t B = so[v == 0 ? 0 : v == 1 ? 2 : 4];   // entry bytes before this round (no commas)
    int64_t C = so[v == 0 ? 1 : v == 1 ? 3 : 5];   // entries before this round
    for (int r0 = s0; r0 < s1; r0 += kJsonWBlock) {
      const int j = r0 + tid;
      int n = 0;
      uint32_t st = 0;
      int64_t u = 0;
      bool e = false;
      if (j < s1) {
        n = a.t.node_order[j];
        st = a.fstatus[(size_t)k * N + n];
        e = st != KSG_FS_NOT_EVALUATED && (v == 0 || st == 0);
        if (e) {
          uint32_t err = 0;
          u = (a.t.node_key_off[n + 1] - a.t.node_key_off[n]) +
              (v == 0 ? filter_body(a, q, st, n, nullptr, err) : score_body(a, q, k, n, v == 2, nullptr));
        }
      }
      int64_t tot;
      const int64_t x = wblock_exscan(((int64_t)e << 40) | u, s_buf, tot);
      const int64_t g = C + (x >> 40);
      const int64_t p = 1 + B + (x & kLow) + g - (g > 0 ? 1 : 0);   // the entry's first byte (its comma)
      const int64_t len = u + (g > 0 ? 1 : 0);
      const int64_t Ce = C + (tot >> 40);
      const int64_t Rlo = 1 + B + C - (C > 0 ? 1 : 0);
      const int64_t Rhi = 1 + B + (tot & kLow) + Ce - (Ce > 0 ? 1 : 0);
      for (int64_t lo = Rlo; lo < Rhi; lo += kJsonWin) {
        const int64_t hi = min(Rhi, lo + (int64_t)kJsonWin);
        if (e && p < hi && p + len > lo) {
          JsonWin w{s_win, lo, hi, p};
          if (g > 0) w.c(',');
          w.s(a.t.node_keys + a.t.node_key_off[n], a.t.node_key_off[n + 1] - a.t.node_key_off[n]);
          if (v == 0)
            emit_filter(w, a, q, st, n);
          else
            emit_score(w, a, q, k, n, v == 2);
        }
        __syncthreads();
        for (int64_t i = tid; i < hi - lo; i += kJsonWBlock) out[lo + i] = s_win[i];
        __syncthreads();
      }
      B += tot & kLow;
      C = Ce;
    }
  }
  if (seg == 0 && tid == 0) {
    for (int v = 0; v < 3; v++) {
      char* const o = a.out + a.offsets[3 * k + v];
      const int64_t l = a.offsets[3 * k + v + 1] - a.offsets[3 * k + v];
      o[0] = '{';
      o[l - 1] = '}';
    }
  }
}

}  // namespace ksk
