// Bulk result-store serialiser, host code in libksched.so.
//
// The wrapped plugins write one map entry per (node, plugin) into
// resultstore.Store under a global mutex (store.go:423 AddFilterResult, :461
// AddScoreResult, :481 AddNormalizedScoreResult), and GetStoredResult
// json.Marshals the maps (store.go:133-198, add*ResultToMap :200-420).  Here
// the three O(N) annotations (filter-result, score-result, finalscore-result)
// are emitted straight from one pod's capture SoA, byte-identical to Go's
// encoding/json output: map keys sorted bytewise, HTML-safe escaping of < > &,
// U+2028/U+2029 escaped, invalid UTF-8 replaced by U+FFFD, \b \f \n \r \t
// short escapes, other control characters as \u00XX.
//
// Output side: each value goes into a raw append buffer kept by the annotator
// (reserved once per node for that node's worst case, then plain stores);
// node keys are escaped once per annotator, a passing node's filter entries
// are one fragment per call, integers are written right to left.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ksched.h"
#include "ksched_json_host.h"

namespace {

void go_string(std::string& o, const char* s) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
  while (*p) {
    const unsigned char c = *p;
    if (c < 0x80) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        case '<': o += "\\u003c"; break;
        case '>': o += "\\u003e"; break;
        case '&': o += "\\u0026"; break;
        default:
          if (c < 0x20) {
            o += "\\u00";
            o.push_back(hex[c >> 4]);
            o.push_back(hex[c & 15]);
          } else {
            o.push_back((char)c);
          }
      }
      p++;
      continue;
    }
    // decode one UTF-8 sequence (utf8.DecodeRuneInString rules)
    int len = 0;
    uint32_t cp = 0, lo = 0;
    if (c >= 0xC2 && c <= 0xDF) { len = 2; cp = c & 0x1F; lo = 0x80; }
    else if (c >= 0xE0 && c <= 0xEF) { len = 3; cp = c & 0x0F; lo = 0x800; }
    else if (c >= 0xF0 && c <= 0xF4) { len = 4; cp = c & 0x07; lo = 0x10000; }
    bool ok = len > 0;
    for (int i = 1; ok && i < len; i++) {
      if ((p[i] & 0xC0) != 0x80) ok = false;
      else cp = (cp << 6) | (p[i] & 0x3F);
    }
    if (ok && (cp < lo || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))) ok = false;
    if (!ok) {
      o += "\xEF\xBF\xBD";   // U+FFFD, one invalid byte consumed
      p++;
      continue;
    }
    if (cp == 0x2028) o += "\\u2028";
    else if (cp == 0x2029) o += "\\u2029";
    else o.append(reinterpret_cast<const char*>(p), len);
    p += len;
  }
  o.push_back('"');
}

const char* kFitRes[3] = {"cpu", "memory", "ephemeral-storage"};

// Fixed-width pieces for the score maps' inner loop: a plugin's key (with the
// separator before it) in a 48-byte slot, and "0" .. "999" quoted in 8-byte
// slots; each is stored whole and the buffer advances by its length (the
// reserve covers the slack).
struct Frag {
  char b[48];
  uint32_t n;
};
struct SmallInt {
  char b[8];
  uint32_t n;
};
// A growable byte buffer without initialisation on growth: reserve() for the
// worst case of what follows, then put() / ch() store without checks.
struct Buf {
  char* d = nullptr;
  size_t n = 0, cap = 0;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { std::free(d); }
  bool reserve(size_t k) {   // room for k more bytes and a terminating NUL
    if (n + k + 1 <= cap) return true;
    const size_t c = std::max(cap * 2, n + k + 1 + ((size_t)1 << 16));
    char* x = static_cast<char*>(std::realloc(d, c));
    if (!x) return false;
    d = x;
    cap = c;
    return true;
  }
  void put(const char* s, size_t k) {
    std::memcpy(d + n, s, k);
    n += k;
  }
  void put(const std::string& s) { put(s.data(), s.size()); }
  void ch(char c) { d[n++] = c; }
  void frag(const Frag& f) {   // 48 bytes stored, f.n kept
    std::memcpy(d + n, f.b, sizeof f.b);
    n += f.n;
  }
  void qint_small(int64_t v, const SmallInt* t) {
    if ((uint64_t)v < 1000) {
      std::memcpy(d + n, t[v].b, sizeof t[v].b);
      n += t[v].n;
    } else {
      qint(v);
    }
  }
  void qint(int64_t v) {   // "<decimal>" (go_int's bytes); at most 22 bytes
    char t[24];
    char* e = t + sizeof t;
    char* q = e;
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do {
      *--q = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    if (v < 0) *--q = '-';
    d[n++] = '"';
    put(q, (size_t)(e - q));
    d[n++] = '"';
  }
};
constexpr size_t kQint = 22;

const SmallInt* small_ints() {
  static const std::vector<SmallInt> t = [] {
    std::vector<SmallInt> v(1000);
    for (int i = 0; i < 1000; i++) {
      const std::string q = "\"" + std::to_string(i) + "\"";
      std::memset(v[i].b, 0, sizeof v[i].b);
      std::memcpy(v[i].b, q.data(), q.size());
      v[i].n = (uint32_t)q.size();
    }
    return v;
  }();
  return t.data();
}

}  // namespace

struct ksg_annotator {
  int32_t N = 0;
  std::vector<std::string> node_json;     // escaped, quoted node names, then ':'
  size_t node_json_max = 0;
  std::vector<int32_t> node_order;        // node indices sorted bytewise by name
  std::string plugin[KSG_NPLUGINS];       // escaped, quoted plugin names, then ':'
  std::string plugin_raw[KSG_NPLUGINS];
  std::vector<std::string> res;           // resource names
  std::vector<std::string> taint;         // "{key: value}" per taint-vocab id
  int32_t max_taints = 0;
  std::vector<uint32_t> taints;           // [max_taints][N]
  Buf out[3];
  std::string pass_all, msg;   // per-call scratch
  // a rejected node's message, JSON-escaped, by status key (the word, plus the
  // taint id for TaintToleration): direct-mapped, valid for one call
  static constexpr int kMsgSlots = 64;
  uint64_t msg_key[kMsgSlots];
  std::string msg_json[kMsgSlots];
};

extern "C" int ksg_annotator_new(const ksg_names* names, ksg_annotator** out) {
  if (!names || !out || names->n_nodes < 0 || (names->n_nodes > 0 && !names->node) || !names->plugin)
    return KSG_E_INVALID;
  ksg_annotator* a = new (std::nothrow) ksg_annotator();
  if (!a) return KSG_E_NOMEM;
  a->N = names->n_nodes;
  a->node_json.resize(a->N);
  a->node_order.resize(a->N);
  for (int i = 0; i < a->N; i++) {
    go_string(a->node_json[i], names->node[i] ? names->node[i] : "");
    a->node_json[i].push_back(':');
    a->node_json_max = std::max(a->node_json_max, a->node_json[i].size());
    a->node_order[i] = i;
  }
  std::stable_sort(a->node_order.begin(), a->node_order.end(), [&](int x, int y) {
    return std::strcmp(names->node[x], names->node[y]) < 0;   // bytewise (unsigned) like Go's string <
  });
  for (int p = 0; p < KSG_NPLUGINS; p++) {
    const char* s = names->plugin[p] ? names->plugin[p] : "";
    a->plugin_raw[p] = s;
    go_string(a->plugin[p], s);
    a->plugin[p].push_back(':');
  }
  for (int r = 0; r < names->n_res; r++) a->res.emplace_back(names->res[r] ? names->res[r] : "");
  for (int t = 0; t < names->n_taint_vocab; t++) a->taint.emplace_back(names->taint[t] ? names->taint[t] : "");
  a->max_taints = names->max_taints;
  if (names->max_taints > 0 && names->taints)
    a->taints.assign(names->taints, names->taints + (size_t)names->max_taints * a->N);
  *out = a;
  return KSG_OK;
}

extern "C" int ksg_annotator_free(ksg_annotator* a) {
  delete a;
  return KSG_OK;
}

namespace {

// framework.py Decoder.message restated: status word -> upstream message.
bool filter_message(const ksg_annotator* a, uint32_t st, int n, std::string& msg) {
  const int pl = (int)(st & 0xFF) - 1;
  const uint32_t reason = st >> 8;
  msg.clear();
  switch (pl) {
    case KSG_PL_NODE_UNSCHEDULABLE: msg = "node(s) were unschedulable"; return true;
    case KSG_PL_NODE_NAME: msg = "node(s) didn't match the requested node name"; return true;
    case KSG_PL_TAINT_TOLERATION: {
      if ((int)reason >= a->max_taints) return false;
      const uint32_t id = a->taints[(size_t)reason * a->N + n];
      if (id == 0 || id > a->taint.size()) return false;
      msg = "node(s) had untolerated taint " + a->taint[id - 1];
      return true;
    }
    case KSG_PL_NODE_AFFINITY: msg = "node(s) didn't match Pod's node affinity/selector"; return true;
    case KSG_PL_NODE_PORTS: msg = "node(s) didn't have free ports for the requested pod ports"; return true;
    case KSG_PL_NODE_RESOURCES_FIT: {
      // noderesources.fitsRequest order: pods, cpu, memory, ephemeral, scalars by column
      bool first = true;
      auto add = [&](const std::string& s) {
        if (!first) msg += ", ";
        msg += s;
        first = false;
      };
      if (reason & 1u) add("Too many pods");
      for (int r = 0; r < (int)a->res.size(); r++)
        if (reason & (1u << (r + 1))) add(std::string("Insufficient ") + (r < 3 ? kFitRes[r] : a->res[r].c_str()));
      return true;
    }
    case KSG_PL_POD_TOPOLOGY_SPREAD:
      msg = reason == 1 ? "node(s) didn't match pod topology spread constraints (missing required label)"
                        : "node(s) didn't match pod topology spread constraints";
      return true;
    case KSG_PL_INTER_POD_AFFINITY:
      if (reason == 1) msg = "node(s) didn't match pod affinity rules";
      else if (reason == 2) msg = "node(s) didn't match pod anti-affinity rules";
      else if (reason == 3) msg = "node(s) didn't satisfy existing pods anti-affinity rules";
      else return false;
      return true;
    case KSG_PL_VOLUME_RESTRICTIONS:
      msg = "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode";
      return true;
    case KSG_PL_VOLUME_BINDING: {   // FindPodVolumes' reason order
      static const char* const kVb[3] = {"node(s) had volume node affinity conflict",
                                         "node(s) didn't find available persistent volumes to bind",
                                         "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)"};
      if (!reason || reason > 7) return false;
      for (int b = 0; b < 3; b++)
        if (reason & (1u << b)) {
          if (!msg.empty()) msg += ", ";
          msg += kVb[b];
        }
      return true;
    }
    case KSG_PL_VOLUME_ZONE:
      msg = "node(s) had no available volume zone";
      return true;
    default:
      return false;
  }
}

std::vector<int> sorted_plugins(const ksg_annotator* a, const int32_t* ids, int n) {
  std::vector<int> v(ids, ids + n);
  std::sort(v.begin(), v.end(), [&](int x, int y) { return a->plugin_raw[x] < a->plugin_raw[y]; });
  return v;
}

}  // namespace

extern "C" int ksg_annotate(ksg_annotator* a, const ksg_annotate_in* in, const char** json, int64_t* len) {
  if (!a || !in || !json || !len || !in->fstatus) return KSG_E_INVALID;
  if (in->n_filter < 0 || in->n_filter > KSG_NPLUGINS || in->n_score < 0 || in->n_score > KSG_NPLUGINS)
    return KSG_E_INVALID;
  for (int i = 0; i < in->n_filter; i++)
    if (in->filter_order[i] < 0 || in->filter_order[i] >= KSG_NPLUGINS) return KSG_E_INVALID;
  for (int i = 0; i < in->n_score; i++)
    if (in->score_order[i] < 0 || in->score_order[i] >= KSG_NPLUGINS) return KSG_E_INVALID;
  const int N = a->N;
  for (auto& b : a->out) b.n = 0;
  // ---- filter-result (store.go:423; nodes outside PreFilterResult absent)
  Buf& f = a->out[0];
  if (!f.reserve(2)) return KSG_E_NOMEM;
  f.ch('{');
  if (in->n_filter > 0) {
    // position of each plugin in run order; a node's entries are the plugins
    // up to and including the first rejecting one
    int pos[KSG_NPLUGINS];
    for (int p = 0; p < KSG_NPLUGINS; p++) pos[p] = -1;
    for (int i = 0; i < in->n_filter; i++) pos[in->filter_order[i]] = i;
    const std::vector<int> by_name = sorted_plugins(a, in->filter_order, in->n_filter);
    for (auto& k : a->msg_key) k = ~0ull;
    // a passing node's entries: every plugin that ran, "passed"
    std::string& pass_all = a->pass_all;
    pass_all.assign(1, '{');
    size_t keys = 0;
    for (int p : by_name) {
      if (pass_all.size() > 1) pass_all.push_back(',');
      pass_all += a->plugin[p];
      pass_all += "\"passed\"";
      keys += a->plugin[p].size() + 1;
    }
    pass_all.push_back('}');
    const size_t pass_bound = a->node_json_max + 1 + pass_all.size();
    bool first_node = true;
    for (int k = 0; k < N; k++) {
      const int n = a->node_order[k];
      const uint32_t st = in->fstatus[n];
      if (st == KSG_FS_NOT_EVALUATED) continue;
      if (st == 0) {
        if (!f.reserve(pass_bound)) return KSG_E_NOMEM;
        if (!first_node) f.ch(',');
        first_node = false;
        f.put(a->node_json[n]);
        f.put(pass_all);
        continue;
      }
      const int fail = (int)(st & 0xFF) - 1;
      const int last = fail < KSG_NPLUGINS ? pos[fail] : -1;
      if (last < 0) return KSG_E_INVALID;   // rejected by a plugin that did not run
      uint64_t key = st;
      if (fail == KSG_PL_TAINT_TOLERATION && (int)(st >> 8) < a->max_taints)
        key |= (uint64_t)a->taints[(size_t)(st >> 8) * N + n] << 32;
      const int slot = (int)((key * 0x9E3779B97F4A7C15ull) >> 58);
      std::string& mj = a->msg_json[slot];
      if (a->msg_key[slot] != key) {
        if (!filter_message(a, st, n, a->msg)) return KSG_E_INVALID;
        mj.clear();
        go_string(mj, a->msg.c_str());
        a->msg_key[slot] = key;
      }
      if (!f.reserve(a->node_json_max + 3 + keys + by_name.size() * 8 + mj.size())) return KSG_E_NOMEM;
      if (!first_node) f.ch(',');
      first_node = false;
      f.put(a->node_json[n]);
      f.ch('{');
      bool first = true;
      for (int p : by_name) {
        if (pos[p] > last) continue;
        if (!first) f.ch(',');
        first = false;
        f.put(a->plugin[p]);
        if (p == fail) f.put(mj);
        else f.put("\"passed\"", 8);
      }
      f.ch('}');
    }
  }
  f.ch('}');
  // ---- score-result / finalscore-result (store.go:461, :481, :504-507)
  Buf& s = a->out[1];
  Buf& t = a->out[2];
  if (!s.reserve(2) || !t.reserve(2)) return KSG_E_NOMEM;
  s.ch('{');
  t.ch('{');
  if (in->n_feasible >= 2 && in->n_score > 0) {
    if (!in->raw || !in->weight) return KSG_E_INVALID;
    const std::vector<int> by_name = sorted_plugins(a, in->score_order, in->n_score);
    // per plugin in key order: its key fragment ("{" or "," before it), its
    // rows and weight
    const int S = (int)by_name.size();
    std::vector<Frag> frag(S);
    std::vector<const int64_t*> raw_row(S), fin_row(S);
    std::vector<uint64_t> wt(S);
    bool fixed = true;
    for (int i = 0; i < S; i++) {
      const int p = by_name[i];
      const std::string key = (i ? "," : "{") + a->plugin[p];
      fixed = fixed && key.size() <= sizeof frag[i].b;
      std::memset(frag[i].b, 0, sizeof frag[i].b);
      std::memcpy(frag[i].b, key.data(), std::min(key.size(), sizeof frag[i].b));
      frag[i].n = (uint32_t)key.size();
      raw_row[i] = in->raw + (size_t)p * N;
      fin_row[i] = ((in->normalize_mask >> p) & 1u) && in->norm ? in->norm + (size_t)p * N : raw_row[i];
      wt[i] = (uint64_t)in->weight[p];
    }
    const SmallInt* small = small_ints();
    size_t bound = a->node_json_max + 3;
    for (int p : by_name) bound += a->plugin[p].size() + 1 + sizeof(Frag{}.b) + kQint + 8;
    bool first_node = true;
    for (int k = 0; k < N; k++) {
      const int n = a->node_order[k];
      if (in->fstatus[n] != 0) continue;
      if (!s.reserve(bound) || !t.reserve(bound)) return KSG_E_NOMEM;
      if (!first_node) { s.ch(','); t.ch(','); }
      first_node = false;
      s.put(a->node_json[n]);
      t.put(a->node_json[n]);
      for (int i = 0; i < S; i++) {
        if (fixed) {
          s.frag(frag[i]);
          t.frag(frag[i]);
        } else {
          const std::string key = (i ? "," : "{") + a->plugin[by_name[i]];
          s.put(key);
          t.put(key);
        }
        const int64_t raw = raw_row[i][n];
        s.qint_small(raw, small);
        const uint64_t v = (uint64_t)fin_row[i][n] * wt[i];
        t.qint_small((int64_t)v, small);   // Go int64 multiplication wraps
      }
      if (S == 0) { s.ch('{'); t.ch('{'); }
      s.ch('}');
      t.ch('}');
    }
  }
  s.ch('}');
  t.ch('}');
  for (int i = 0; i < 3; i++) {
    a->out[i].d[a->out[i].n] = 0;
    json[i] = a->out[i].d;
    len[i] = (int64_t)a->out[i].n;
  }
  return KSG_OK;
}

// The device serialiser's tables (ksched_json.h): the same escaped pieces
// this file's ksg_annotate writes, packed flat.
int ksg_annotator_json_tables(const ksg_annotator* a, JsonHostTables* t) {
  if (!a || !t) return KSG_E_INVALID;
  const int N = a->N;
  t->node_keys.clear();
  t->node_key_off.assign(1, 0);
  for (int n = 0; n < N; n++) {
    t->node_keys += a->node_json[n];
    t->node_key_off.push_back((int64_t)t->node_keys.size());
  }
  t->node_order = a->node_order;
  t->plugin_keys.clear();
  t->plugin_key_off.assign(1, 0);
  for (int p = 0; p < KSG_NPLUGINS; p++) {
    t->plugin_keys += a->plugin[p];
    t->plugin_key_off.push_back((int32_t)t->plugin_keys.size());
  }
  int ids[KSG_NPLUGINS];
  for (int p = 0; p < KSG_NPLUGINS; p++) ids[p] = p;
  const std::vector<int> order = sorted_plugins(a, ids, KSG_NPLUGINS);
  for (int i = 0; i < KSG_NPLUGINS; i++) t->by_name[i] = order[i];
  // the messages that depend on nothing but (plugin, reason)
  t->msgs.clear();
  t->msg_off.assign(1, 0);
  std::string m, q;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    for (int r = 0; r < 8; r++) {
      if (pl != KSG_PL_TAINT_TOLERATION && pl != KSG_PL_NODE_RESOURCES_FIT &&
          filter_message(a, (uint32_t)(pl + 1) | ((uint32_t)r << 8), 0, m)) {
        q.clear();
        go_string(q, m.c_str());
        t->msgs += q;
      }
      t->msg_off.push_back((int32_t)t->msgs.size());
    }
  t->taint_msgs.clear();
  t->taint_msg_off.assign(1, 0);
  for (auto& tn : a->taint) {
    q.clear();
    go_string(q, ("node(s) had untolerated taint " + tn).c_str());
    t->taint_msgs += q;
    t->taint_msg_off.push_back((int32_t)t->taint_msgs.size());
  }
  auto inner = [&](const std::string& x) {   // escaped, without the quotes
    q.clear();
    go_string(q, x.c_str());
    return q.substr(1, q.size() - 2);
  };
  t->fit_parts = inner("Too many pods");
  t->fit_part_off.assign(1, 0);
  t->fit_part_off.push_back((int32_t)t->fit_parts.size());
  for (int r = 0; r < (int)a->res.size(); r++) {
    t->fit_parts += inner(std::string("Insufficient ") + (r < 3 ? kFitRes[r] : a->res[r].c_str()));
    t->fit_part_off.push_back((int32_t)t->fit_parts.size());
  }
  t->n_res = (int32_t)a->res.size();
  t->n_taint_vocab = (int32_t)a->taint.size();
  t->max_taints = a->max_taints;
  return KSG_OK;
}
