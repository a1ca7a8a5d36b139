// Native snapshot encoder (include/ksched_snapshot.h): NodeInfo / PodInfo
// views -> the SoA columns, interned ids and compiled selector programs of
// include/ksched.h.  Host code only (no device needed), part of libksched.so.
//
// The encoding is the one encoder.py documents (program grammar in its module
// docstring); the two are independent restatements of the same contract and
// tests/test_snapshot_native.py requires byte-identical output from both on
// every workload family.  Upstream semantics restated here [upstream
// k8s.io/kubernetes v1.32.5, not vendored — SURVEY.md §8(c)]:
//   resourcehelper.PodRequests (non-missing cpu/memory defaults for the
//   non-zero form), v1.Toleration.ToleratesTaint,
//   metav1.LabelSelectorAsSelector, podtopologyspread
//   filterTopologySpreadConstraints / buildDefaultConstraints,
//   framework.AffinityTerm namespaces, imagelocality normalizedImageName and
//   scaledImageScore, nodeaffinity PreFilter (matchFields metadata.name ->
//   PreFilterResult), Go math.Log (src/math/log.go).
// The framework.Status codes returned by ksg_snapshot_status follow the
// plugins' Filter returns.
#include "ksched_snapshot.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <emmintrin.h>   // SSE2 (x86-64 baseline): ksg_snapshot_statuses
#include <iterator>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

// ---- plugin table (profile.py) ----------------------------------------------
const char* const kPluginNames[KSG_NPLUGINS] = {
    "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
    "NodeResourcesFit", "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding",
    "VolumeZone", "PodTopologySpread", "InterPodAffinity",
    "NodeResourcesBalancedAllocation", "ImageLocality"};
// extension points per plugin: prefilter, filter, prescore, score, normalize
const bool kExt[KSG_NPLUGINS][5] = {
    {false, true, false, false, false}, {false, true, false, false, false}, {false, true, true, true, true},
    {true, true, true, true, true},     {true, true, false, false, false},  {true, true, true, true, false},
    {true, true, false, false, false},  {true, true, false, false, false},  {true, true, true, true, false},
    {true, true, false, false, false},  {true, true, true, true, true},     {true, true, true, true, true},
    {false, false, true, true, false},  {false, false, false, true, false}};
const char* const kNonEval[] = {"SchedulingGates", "PrioritySort", "DefaultPreemption", "DefaultBinder"};

const std::string kCPU = "cpu", kMemory = "memory", kEphemeral = "ephemeral-storage", kPods = "pods";
const std::string kHostname = "kubernetes.io/hostname", kZone = "topology.kubernetes.io/zone";
const std::string kObjectName = "metadata.name";
const std::string kBindAllHostIP = "0.0.0.0";   // framework.DefaultBindAllHostIP
const std::string kUnschedTaint = "node.kubernetes.io/unschedulable";
constexpr int64_t kDefaultMilliCPU = 100, kDefaultMemory = 200ll * 1024 * 1024;

enum { OP_IN = 0, OP_NOT_IN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_NEVER };
enum { TMPL_REQ_ANTI = 0, TMPL_REQ_AFF = 1, TMPL_PREF = 2 };

int op_code(const std::string& s) {
  if (s == "In") return OP_IN;
  if (s == "NotIn") return OP_NOT_IN;
  if (s == "Exists") return OP_EXISTS;
  if (s == "DoesNotExist") return OP_DNE;
  if (s == "Gt") return OP_GT;
  if (s == "Lt") return OP_LT;
  return -1;
}

int effect_code(const std::string& e) {
  return e == "NoSchedule" ? KSG_EFFECT_NO_SCHEDULE
         : e == "PreferNoSchedule" ? KSG_EFFECT_PREFER_NO_SCHEDULE
         : e == "NoExecute" ? KSG_EFFECT_NO_EXECUTE : 0;
}

std::string S(const char* p) { return p ? std::string(p) : std::string(); }

bool starts_with(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

// schedutil.IsScalarResourceName
bool is_scalar(const std::string& n) {
  if (starts_with(n, "hugepages-") || starts_with(n, "attachable-volumes-")) return true;
  return n.find('/') != std::string::npos && !starts_with(n, "kubernetes.io/") && !starts_with(n, "requests.");
}

// strconv.ParseInt(s, 10, 64)
bool parse_int64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = (s[0] == '+' || s[0] == '-') ? 1 : 0;
  if (i == s.size()) return false;
  const bool neg = s[0] == '-';
  unsigned long long v = 0;
  const unsigned long long lim = neg ? (1ull << 63) : (1ull << 63) - 1;
  for (; i < s.size(); i++) {
    const char ch = s[i];
    if (ch < '0' || ch > '9') return false;
    const unsigned d = ch - '0';
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

// Go math.Log (src/math/log.go; FreeBSD e_log.c).  Built with
// -ffp-contract=off: Go on amd64 does not fuse.
double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || (std::isinf(x) && x > 0)) return x;
  if (x < 0) return std::nan("");
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < std::sqrt(2.0) / 2) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1, k = (double)ki;
  const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2, hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

int32_t s32(uint64_t x) { return (int32_t)(uint32_t)(x & 0xffffffffu); }

// ---- object model (copies of the views) --------------------------------------
using StrMap = std::map<std::string, std::string>;
using ResMap = std::map<std::string, int64_t>;

struct Req {
  std::string key, op;
  std::vector<std::string> values;
};
struct Sel {
  bool set = false;
  std::vector<std::pair<std::string, std::string>> labels;
  std::vector<Req> expr;
  bool empty() const { return labels.empty() && expr.empty(); }
};
struct Term {
  std::vector<Req> expr, fields;
};
struct PrefTerm {
  int32_t weight;
  Term pref;
};
struct AffTerm {
  int32_t weight;
  Sel sel;
  std::string key;
  std::vector<std::string> ns;
  Sel ns_sel;
  // a namespaceSelector with requirements, as given: resolved into `ns`
  // against the snapshot's namespaces (ns_given ∪ matching namespaces)
  bool resolved = false;
  std::vector<std::string> ns_given;
  Sel ns_req;
};
// A namespace no pod can have: a resolved namespaceSelector that matched
// nothing (ingest.py NO_NAMESPACE).
const std::string kNoNamespace = std::string("\0none", 5);
struct Spread {
  int32_t skew, min_domains;
  std::string key, when, nap, ntp;
  Sel sel;
  std::vector<std::string> mlk;
};
// sanitised (hostIP, protocol, hostPort): framework.HostPortInfo's key
using HostPort = std::tuple<std::string, std::string, int32_t>;
struct Container {
  std::string image;
  ResMap req;
  bool restartable;
  std::vector<HostPort> host_ports;   // hostPort > 0 only
};
struct Taint {
  std::string key, value, effect;
  bool operator<(const Taint& o) const { return std::tie(key, value, effect) < std::tie(o.key, o.value, o.effect); }
};
struct Tol {
  std::string key, op, value, effect;
  // v1.Toleration.ToleratesTaint
  bool tolerates(const Taint& t) const {
    if (!effect.empty() && effect != t.effect) return false;
    if (!key.empty() && key != t.key) return false;
    if (op.empty() || op == "Equal") return value == t.value;
    return op == "Exists";
  }
};
struct Image {
  std::vector<std::string> names;
  int64_t size;
};
struct Node {
  std::string name;
  StrMap labels;
  std::vector<Taint> taints;
  ResMap alloc;
  bool unsched;
  std::vector<Image> images;
};
// The volume plugins' objects [upstream v1.32 volumebinding / volumezone /
// volumerestrictions listers; model.py PersistentVolume / Claim / StorageClass]
struct PV {
  std::string name;
  StrMap labels;
  std::string storage_class;
  bool has_claim_ref = false;
  std::string claim_ns, claim_name;
  std::string source;
  bool has_na = false;
  std::vector<Term> na;
};
struct PVC {
  std::string ns, name, volume_name, storage_class;
  std::vector<std::string> modes;
  StrMap ann;
  bool deleting = false;
  // volumeBinder.isPVCFullyBound: a volume name and bind-completed
  bool fully_bound() const { return !volume_name.empty() && ann.count("pv.kubernetes.io/bind-completed"); }
};
struct SClass {
  std::string name, provisioner, mode;
  std::vector<std::vector<std::pair<std::string, std::vector<std::string>>>> topo;   // allowedTopologies
};
const char* const kZoneLabels[4] = {"failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                                    "topology.kubernetes.io/zone", "topology.kubernetes.io/region"};
std::string ga_label(const std::string& k) {   // volumezone translateToGALabel
  if (k == kZoneLabels[0]) return kZoneLabels[2];
  if (k == kZoneLabels[1]) return kZoneLabels[3];
  return k;
}
const std::string kWFFC = "WaitForFirstConsumer";
constexpr int32_t kVolRwopConflict = 1;   // VolumeRestrictions rejects every node (encoder.py VOL_RWOP_CONFLICT)

struct Pod {
  std::string ns, name, node_name;
  StrMap labels;
  std::vector<Container> containers, init;
  bool has_overhead;
  ResMap overhead;
  bool has_node_selector, has_na_req, has_na_pref;
  StrMap node_selector;
  std::vector<Term> na_req;
  std::vector<PrefTerm> na_pref;
  std::vector<AffTerm> aff_req, aff_pref, anti_req, anti_pref;
  std::vector<Tol> tols;
  std::vector<Spread> spread;
  Sel default_sel;
  bool terminating;
  int32_t priority;
  std::vector<std::string> claims;   // spec.volumes[].persistentVolumeClaim.claimName, in volume order
};

std::vector<Req> copy_reqs(int32_t n, const ksg_requirement_view* v) {
  std::vector<Req> out;
  for (int32_t i = 0; i < n; i++) {
    Req r{S(v[i].key), S(v[i].op), {}};
    for (int32_t k = 0; k < v[i].n_values; k++) r.values.push_back(S(v[i].values[k]));
    out.push_back(std::move(r));
  }
  return out;
}
Sel copy_sel(const ksg_label_selector_view& v) {
  Sel s;
  s.set = v.is_set != 0;
  if (!s.set) return s;
  for (int32_t i = 0; i < v.n_labels; i++) s.labels.emplace_back(S(v.match_labels[i].key), S(v.match_labels[i].value));
  s.expr = copy_reqs(v.n_expr, v.expr);
  return s;
}
Term copy_term(const ksg_node_selector_term_view& v) {
  return Term{copy_reqs(v.n_expr, v.expr), copy_reqs(v.n_fields, v.fields)};
}
StrMap copy_pairs(int32_t n, const ksg_str_pair* p) {
  StrMap m;
  for (int32_t i = 0; i < n; i++) m[S(p[i].key)] = S(p[i].value);
  return m;
}
ResMap copy_res(int32_t n, const ksg_quantity* q) {
  ResMap m;
  for (int32_t i = 0; i < n; i++) m[S(q[i].name)] = q[i].value;
  return m;
}
std::vector<AffTerm> copy_aff(int32_t n, const ksg_affinity_term_view* v) {
  std::vector<AffTerm> out;
  for (int32_t i = 0; i < n; i++) {
    AffTerm t;
    t.weight = v[i].weight;
    t.sel = copy_sel(v[i].selector);
    t.key = S(v[i].topology_key);
    for (int32_t k = 0; k < v[i].n_namespaces; k++) t.ns.push_back(S(v[i].namespaces[k]));
    t.ns_sel = copy_sel(v[i].namespace_selector);
    out.push_back(std::move(t));
  }
  return out;
}
std::vector<Container> copy_containers(int32_t n, const ksg_container_view* v) {
  std::vector<Container> out;
  for (int32_t i = 0; i < n; i++) {
    Container c{S(v[i].image), copy_res(v[i].n_requests, v[i].requests), v[i].restartable != 0, {}};
    for (int32_t k = 0; k < v[i].n_host_ports; k++) {
      const ksg_host_port_view& hp = v[i].host_ports[k];
      if (hp.host_port <= 0) continue;   // GetHostPorts: only ports with a hostPort
      std::string ip = S(hp.host_ip), proto = S(hp.protocol);
      c.host_ports.emplace_back(ip.empty() ? kBindAllHostIP : ip, proto.empty() ? "TCP" : proto, hp.host_port);
    }
    out.push_back(std::move(c));
  }
  return out;
}

// schedutil.GetHostPorts: restartable init containers, then the containers
std::vector<HostPort> pod_host_ports(const Pod& p) {
  std::vector<HostPort> out;
  for (auto& c : p.init)
    if (c.restartable) out.insert(out.end(), c.host_ports.begin(), c.host_ports.end());
  for (auto& c : p.containers) out.insert(out.end(), c.host_ports.begin(), c.host_ports.end());
  return out;
}

// ---- resourcehelper.PodRequests -------------------------------------------------
void add_to(ResMap& d, const ResMap& s) {
  for (auto& kv : s) d[kv.first] += kv.second;
}
void max_to(ResMap& d, const ResMap& s) {
  for (auto& kv : s) {
    auto it = d.find(kv.first);
    if (it == d.end() || kv.second > it->second) d[kv.first] = kv.second;
  }
}
ResMap non_missing(const ResMap& r, bool nz) {
  ResMap cp = r;
  if (nz) {
    if (!r.count(kCPU)) cp[kCPU] += kDefaultMilliCPU;
    if (!r.count(kMemory)) cp[kMemory] += kDefaultMemory;
  }
  return cp;
}
ResMap pod_requests(const Pod& p, bool nz) {
  ResMap reqs, restartable, init_reqs;
  for (auto& c : p.containers) add_to(reqs, non_missing(c.req, nz));
  for (auto& c : p.init) {
    ResMap cr = non_missing(c.req, nz);
    if (c.restartable) {
      add_to(reqs, cr);
      add_to(restartable, cr);
      cr = restartable;
    } else {
      ResMap tmp;
      add_to(tmp, cr);
      add_to(tmp, restartable);
      cr = tmp;
    }
    max_to(init_reqs, cr);
  }
  max_to(reqs, init_reqs);
  if (p.has_overhead) add_to(reqs, p.overhead);
  return reqs;
}

std::string normalized_image(std::string n) {
  const auto c = n.rfind(':'), s = n.rfind('/');
  const long ci = c == std::string::npos ? -1 : (long)c, si = s == std::string::npos ? -1 : (long)s;
  if (ci <= si) n += ":latest";
  return n;
}

// ---- canonical selectors (encoder.canon_selector) ---------------------------------
using CReq = std::tuple<std::string, int, std::vector<std::string>>;
using Canon = std::optional<std::vector<CReq>>;   // nullopt = labels.Nothing()

struct EncodeError {
  int code;
  std::string msg;
};

Canon canon_selector(const Sel& ls, const StrMap* extra = nullptr) {
  if (!ls.set) return std::nullopt;
  std::set<CReq> reqs;
  for (auto& kv : ls.labels) reqs.insert(CReq{kv.first, OP_IN, {kv.second}});
  for (auto& r : ls.expr) {
    const int op = op_code(r.op);
    if (op < 0) throw EncodeError{KSG_E_INVALID, "label selector operator " + r.op};
    std::set<std::string> vs(r.values.begin(), r.values.end());
    reqs.insert(CReq{r.key, op, std::vector<std::string>(vs.begin(), vs.end())});
  }
  if (extra)
    for (auto& kv : *extra) reqs.insert(CReq{kv.first, OP_IN, {kv.second}});
  return std::vector<CReq>(reqs.begin(), reqs.end());
}

bool reqs_match(const std::vector<CReq>& reqs, const StrMap& labels);
bool selector_matches(const Canon& c, const StrMap& labels) { return c && reqs_match(*c, labels); }
// a canonical selector's requirements (labels.Selector.Matches)
bool reqs_match(const std::vector<CReq>& reqs, const StrMap& labels) {
  for (auto& r : reqs) {
    const auto it = labels.find(std::get<0>(r));
    const bool has = it != labels.end();
    const auto& vals = std::get<2>(r);
    switch (std::get<1>(r)) {
      case OP_IN:
        if (!has || !std::binary_search(vals.begin(), vals.end(), it->second)) return false;
        break;
      case OP_NOT_IN:
        if (has && std::binary_search(vals.begin(), vals.end(), it->second)) return false;
        break;
      case OP_EXISTS:
        if (!has) return false;
        break;
      case OP_DNE:
        if (has) return false;
        break;
      default:
        return false;
    }
  }
  return true;
}

// framework.AffinityTerm scope: (selector, namespaces, all namespaces)
struct Scope {
  Canon canon;
  std::vector<std::string> ns;
  bool ns_all;
  bool operator<(const Scope& o) const { return std::tie(canon, ns, ns_all) < std::tie(o.canon, o.ns, o.ns_all); }
  bool operator==(const Scope& o) const { return canon == o.canon && ns == o.ns && ns_all == o.ns_all; }
  bool ns_match(const std::string& n) const { return ns_all || std::binary_search(ns.begin(), ns.end(), n); }
};

Scope term_scope(const AffTerm& t, const Pod& owner) {
  if (t.ns_sel.set && !t.ns_sel.empty())   // add_pod resolves these (resolve_namespaces)
    throw EncodeError{KSG_E_UNSUPPORTED, "namespaceSelector with requirements needs the snapshot's namespaces"};
  Scope s;
  s.canon = canon_selector(t.sel);
  s.ns_all = t.ns_sel.set;
  std::set<std::string> ns(t.ns.begin(), t.ns.end());
  s.ns.assign(ns.begin(), ns.end());
  if (t.ns.empty() && !t.ns_sel.set) s.ns = {owner.ns};
  return s;
}

// (max_skew, key, canon, min_domains, na_honor, nt_honor)
struct Constraint {
  int32_t skew;
  std::string key;
  Canon canon;
  int32_t min_domains;
  bool na_honor, nt_honor;
};

// ---- the encoded snapshot ---------------------------------------------------------
struct Encoded {
  std::vector<std::string> res_names, label_cols;
  std::map<std::string, int> res_col, col_index;
  std::vector<std::map<std::string, int32_t>> vocab;   // per label column
  std::vector<Taint> taint_vocab;
  std::map<Taint, int> taint_id;
  std::vector<std::string> image_vocab;
  std::map<std::string, int> image_id;
  std::vector<HostPort> port_vocab;    // every host port a pod uses, sorted
  std::map<HostPort, int> port_id;
  std::map<std::string, std::pair<int64_t, int64_t>> image_state;   // name -> (size, numNodes)
  int max_taints = 1, max_images = 1, tol_words = 1;
  // topology universe
  std::map<std::pair<std::vector<CReq>, std::string>, int> pts_sel;
  std::vector<std::pair<std::vector<CReq>, std::string>> pts_order;
  std::map<std::vector<Scope>, int> ipa_sel;   // ids offset by n_pts
  std::vector<std::vector<Scope>> ipa_order;
  std::map<std::tuple<int, Scope, int>, int> templates;
  std::vector<std::tuple<int, Scope, int>> tmpl_order;
  int n_selectors = 0;
  // arrays
  std::vector<int64_t> alloc, requested, nonzero, label_num;
  std::vector<int32_t> allowed, pod_count;
  std::vector<uint8_t> unsched, label_num_ok, taint_effect, col_unique;
  std::vector<uint32_t> label_val, taints, images;
  std::vector<int32_t> col_vocab, tmpl_col, tmpl_kind, tmpl_weight;
  std::vector<double> log_table;
  std::vector<ksg_pod> pods;
  std::vector<int32_t> prog;            // program pool (the views hand out {0} when empty)
  // PreFilter outcomes per pod (profile order, encode_pod): the
  // PreFilterResult node names per plugin (NodeAffinity, VolumeBinding) and
  // the rejecting plugin with its message ("" = the framework's own rejection
  // of an empty intersection)
  std::map<int, std::map<int, std::vector<std::string>>> prefilter_names;
  std::map<int, std::pair<int, std::string>> prefilter_reject;
  std::vector<std::string> taint_strings;
  ksg_profile prof{};
  int N = 0;
};

struct Profile {
  std::vector<std::pair<std::string, int32_t>> plugins;
  std::string fit_strategy;
  std::vector<std::pair<std::string, int64_t>> fit_res, ba_res;
  std::set<std::string> ignored, ignored_groups;
  int32_t hard_weight;
  bool ignore_pref, pts_system, ba_skip_be;
  std::vector<std::pair<int32_t, int32_t>> shape;   // RequestedToCapacityRatio (utilization, score 0..10)
  std::vector<Spread> pts_defaults;                 // defaultConstraints (defaultingType List)
  std::vector<int> enabled;   // plugin ids in MultiPoint order
  // derived (profile.py Profile._expand / weights / selection_weights)
  std::vector<int> order[KSG_NPOINTS];   // per extension point, run order
  int64_t store_w[KSG_NPLUGINS] = {};    // getScorePluginWeight, 0 = absent
  int32_t sel_w[KSG_NPLUGINS] = {};      // the framework's Score weights, 0 = absent
};

}  // namespace

struct ksg_snapshot {
  std::string err;
  Profile prof;
  std::vector<Node> nodes;
  std::map<std::string, int> node_index;
  std::vector<Pod> pods;
  // pods the caller expects to add later (pending in the scheduling queue):
  // their selectors, term templates, label keys, scalar resources and host
  // ports join the encoding universe now, so adding them later appends in
  // place instead of re-encoding (ksg_snapshot_hint_pod).  No program, no
  // binding: they are not pods of the workload.
  std::vector<Pod> hints;
  size_t hints_seen = 0;            // hints[0, hints_seen) are inside the current encoding universe
  std::unordered_map<std::string, size_t> hint_index;   // "ns/name" -> index in hints
  std::vector<std::pair<int32_t, int32_t>> binds;   // (pod, node) in order: bound, then assumed
  Encoded e;
  bool encoded = false;     // e reflects nodes and pods [0, n_encoded)
  int n_encoded = 0;
  int epoch = 0;                    // bumped by every full encode
  ksg_ctx* loaded_ctx = nullptr;   // the context e was last loaded into
  int loaded_epoch = -1;            // the encoding that context holds
  int n_loaded = 0;                 // pods on that context's workload
  size_t prog_loaded = 0;           // program words on that context
  // per-pod encode caches (full encode)
  std::vector<std::pair<std::vector<Constraint>, std::vector<Constraint>>> pts_cache;
  std::vector<std::vector<int>> pod_selectors;
  std::vector<std::vector<std::pair<int, int>>> owned_templates;
  std::vector<std::array<std::vector<int>, 3>> tmpl_match;
  std::vector<std::pair<ResMap, ResMap>> req_cache;
  // views handed out
  std::vector<const char*> v_nodes, v_res, v_taints;
  // scalar resource names of the nodes, pods and profile so far (add_pod
  // refuses a pod that would push the resource columns past KSG_MAX_RES)
  std::set<std::string> scalars;
  // namespaces and their labels (ksg_snapshot_add_namespace): namespaceSelector
  // terms resolve against these
  bool have_namespaces = false;
  std::map<std::string, StrMap> namespaces;
  // the volume plugins' listers (ksg_snapshot_add_pv / _add_pvc / _add_storage_class)
  std::map<std::string, PV> pvs;
  std::map<std::pair<std::string, std::string>, PVC> pvcs;
  std::map<std::string, SClass> classes;
  std::map<std::pair<std::string, std::string>, std::set<int>> claim_users;   // full encode: (ns, claim) -> pods
  std::set<int> bound_set;          // full encode: pods with a binding (running or assumed)
  // match_pod's inverted index of the universe (rebuilt at every full
  // encode): selector / template ids by one (key, value) their match needs;
  // the rest (no In requirement, or matching everything) are scanned
  struct SelIndex {
    std::map<std::pair<std::string, std::string>, std::vector<int>> kv[3];   // pts, ipa, templates
    std::vector<int> scan[3];
  } sel_index;
  bool vol_run = false;             // a volume plugin runs at PreFilter or Filter
  bool csi_limits = false;          // NodeVolumeLimits runs and a node publishes CSI attach limits
  // ksg_snapshot_statuses: a status key's (code, message) is kept across
  // pods until the next full encode (status_epoch); per call, stamp/local
  // number the keys a pod meets in first-seen order
  struct StatusCache {
    int epoch = -1;
    std::unordered_map<uint64_t, int32_t> ids;   // key -> id
    std::vector<std::string> msgs;
    std::vector<int32_t> codes;
    std::vector<uint32_t> stamp;
    std::vector<int32_t> local;
    std::vector<int32_t> order;   // this call's ids, first-seen order
    uint32_t gen = 0;
    static constexpr int kDm = 256;   // direct-mapped front of `ids`
    uint64_t dm_key[kDm];
    int32_t dm_id[kDm];
  } status;
  // ksg_snapshot_statuses_kept: the arrays it returns (owned here, read-only
  // to the caller), whether they hold the last call's complete output, and
  // the nodes that call rejected (the only entries other than Success / -1)
  struct StatusKept {
    std::vector<int32_t> code, msg;
    bool valid = false;
    std::vector<int32_t> rej;
    int64_t sparse_calls = 0, dense_calls = 0;
  } skept;
};

namespace {

int fail(ksg_snapshot* s, int code, const std::string& m) {
  if (s) s->err = m;
  return code;
}

// PodTopologySpread constraints of a pod (encoder._pts_constraints)
using PtsPair = std::pair<std::vector<Constraint>, std::vector<Constraint>>;   // (hard, soft)
PtsPair pts_constraints(const Pod& p, const Profile& prof) {
  std::vector<Constraint> hard, soft;
  if (!p.spread.empty()) {
    for (auto& c : p.spread) {
      StrMap extra;
      for (auto& k : c.mlk) {
        auto it = p.labels.find(k);
        if (it != p.labels.end()) extra[k] = it->second;
      }
      Constraint ent{c.skew, c.key, canon_selector(c.sel, extra.empty() ? nullptr : &extra),
                     c.min_domains > 0 ? c.min_domains : 1, c.nap.empty() || c.nap == "Honor",
                     !c.ntp.empty() && c.ntp == "Honor"};
      if (c.when == "DoNotSchedule") hard.push_back(ent);
      else if (c.when == "ScheduleAnyway") soft.push_back(ent);
    }
  } else if (p.default_sel.set) {   // buildDefaultConstraints with the owners' selector
    Canon canon = canon_selector(p.default_sel);
    if (canon && !canon->empty()) {
      if (prof.pts_system) {
        soft.push_back(Constraint{3, kHostname, canon, 1, true, false});
        soft.push_back(Constraint{5, kZone, canon, 1, true, false});
      } else {
        for (auto& c : prof.pts_defaults) {
          Constraint ent{c.skew, c.key, canon, c.min_domains > 0 ? c.min_domains : 1,
                         c.nap.empty() || c.nap == "Honor", !c.ntp.empty() && c.ntp == "Honor"};
          (c.when == "DoNotSchedule" ? hard : soft).push_back(ent);
        }
      }
    }
  }
  return {hard, soft};
}

// Encoding context of one pass: full (may extend the universe) or frozen
// (an appended pod: any new column / value / selector / template sets miss).
struct Pass {
  ksg_snapshot* s;
  bool frozen;
  bool miss = false;
  Encoded& e() { return s->e; }

  int col(const std::string& key) {
    auto it = e().col_index.find(key);
    if (it == e().col_index.end()) {
      miss = true;
      return 0;
    }
    return it->second;
  }
  int32_t value_id(int c, const std::string& v) {
    auto& voc = e().vocab[c];
    auto it = voc.find(v);
    if (it != voc.end()) return it->second;
    if (frozen) {
      miss = true;
      return 0;
    }
    const int32_t id = (int32_t)voc.size() + 1;
    voc[v] = id;
    return id;
  }
  void emit(std::vector<int32_t>& out, const std::vector<int32_t>& w) { out.insert(out.end(), w.begin(), w.end()); }

  std::vector<int32_t> requirement(const Req& r, bool field) {
    int c;
    if (field) {
      if (r.key != kObjectName || (r.op != "In" && r.op != "NotIn") || r.values.size() != 1) return {0, OP_NEVER, 0};
      c = col(kObjectName);
    } else {
      c = col(r.key);
    }
    if (miss) return {0, OP_NEVER, 0};
    const int op = op_code(r.op);
    if (op < 0) return {0, OP_NEVER, 0};
    if (op == OP_IN || op == OP_NOT_IN) {
      if (r.values.empty()) return {0, OP_NEVER, 0};
      std::set<int32_t> ids;
      for (auto& v : r.values) ids.insert(value_id(c, v));
      std::vector<int32_t> out = {c, op, (int32_t)ids.size()};
      out.insert(out.end(), ids.begin(), ids.end());
      return out;
    }
    if (op == OP_EXISTS || op == OP_DNE) {
      if (!r.values.empty()) return {0, OP_NEVER, 0};
      return {c, op, 0};
    }
    int64_t v;
    if (r.values.size() != 1 || !parse_int64(r.values[0], &v)) return {0, OP_NEVER, 0};
    const uint64_t u = (uint64_t)v;
    return {c, op, 2, s32(u), s32(u >> 32)};
  }
  std::vector<int32_t> term(const Term& t) {
    std::vector<std::vector<int32_t>> reqs;
    for (auto& r : t.expr) reqs.push_back(requirement(r, false));
    for (auto& r : t.fields) reqs.push_back(requirement(r, true));
    std::vector<int32_t> out = {(int32_t)reqs.size()};
    for (auto& r : reqs) emit(out, r);
    return out;
  }
};

// ---- universe (full encode) ---------------------------------------------------
void build_resources(ksg_snapshot* s) {
  Encoded& e = s->e;
  std::set<std::string> scal;
  for (auto& n : s->nodes)
    for (auto& kv : n.alloc)
      if (is_scalar(kv.first)) scal.insert(kv.first);
  s->req_cache.clear();
  for (auto& p : s->pods) {
    s->req_cache.emplace_back(pod_requests(p, false), pod_requests(p, true));
    for (auto& kv : s->req_cache.back().first)
      if (is_scalar(kv.first)) scal.insert(kv.first);
  }
  for (auto& h : s->hints)
    for (auto& kv : pod_requests(h, false))
      if (is_scalar(kv.first)) scal.insert(kv.first);
  for (auto& r : s->prof.fit_res)
    if (is_scalar(r.first)) scal.insert(r.first);
  for (auto& r : s->prof.ba_res)
    if (is_scalar(r.first)) scal.insert(r.first);
  e.res_names = {kCPU, kMemory, kEphemeral};
  e.res_names.insert(e.res_names.end(), scal.begin(), scal.end());
  if ((int)e.res_names.size() > KSG_MAX_RES)
    throw EncodeError{KSG_E_UNSUPPORTED, "more than " + std::to_string(KSG_MAX_RES) + " resource columns"};
  e.res_col.clear();
  for (size_t i = 0; i < e.res_names.size(); i++) e.res_col[e.res_names[i]] = (int)i;
}

// Node label keys a pod's volume program reads (encoder.py
// _volume_label_keys): the zone labels, its bound PVs' node-affinity keys,
// its classes' allowedTopologies keys.
void volume_label_keys(const ksg_snapshot* s, const Pod& p, std::set<std::string>& keys) {
  if (p.claims.empty()) return;
  for (const char* k : kZoneLabels) keys.insert(k);
  for (auto& c : p.claims) {
    auto it = s->pvcs.find({p.ns, c});
    if (it == s->pvcs.end()) continue;
    const PVC& pvc = it->second;
    if (!pvc.volume_name.empty()) {
      auto pt = s->pvs.find(pvc.volume_name);
      if (pt != s->pvs.end() && pt->second.has_na)
        for (auto& t : pt->second.na)
          for (auto& r : t.expr) keys.insert(r.key);
    }
    if (!pvc.storage_class.empty()) {
      auto ct = s->classes.find(pvc.storage_class);
      if (ct != s->classes.end())
        for (auto& term : ct->second.topo)
          for (auto& kv : term) keys.insert(kv.first);
    }
  }
}

void build_label_columns(ksg_snapshot* s) {
  Encoded& e = s->e;
  std::set<std::string> keys;
  bool name_field = false;
  s->pts_cache.clear();
  auto pod_keys = [&](const Pod& p, const PtsPair& pts) {
    if (p.has_node_selector)
      for (auto& kv : p.node_selector) keys.insert(kv.first);
    if (p.has_na_req)
      for (auto& t : p.na_req) {
        for (auto& r : t.expr) keys.insert(r.key);
        name_field |= !t.fields.empty();
      }
    if (p.has_na_pref)
      for (auto& pt : p.na_pref) {
        for (auto& r : pt.pref.expr) keys.insert(r.key);
        name_field |= !pt.pref.fields.empty();
      }
    for (auto& c : pts.first) keys.insert(c.key);
    for (auto& c : pts.second) keys.insert(c.key);
    for (auto* v : {&p.aff_req, &p.anti_req, &p.aff_pref, &p.anti_pref})
      for (auto& t : *v) keys.insert(t.key);
    volume_label_keys(s, p, keys);
  };
  for (auto& p : s->pods) {
    s->pts_cache.push_back(pts_constraints(p, s->prof));
    pod_keys(p, s->pts_cache.back());
  }
  for (auto& h : s->hints) pod_keys(h, pts_constraints(h, s->prof));
  e.label_cols.assign(keys.begin(), keys.end());
  if (name_field) e.label_cols.push_back(kObjectName);
  e.col_index.clear();
  for (size_t i = 0; i < e.label_cols.size(); i++) e.col_index[e.label_cols[i]] = (int)i;
  const size_t L = e.label_cols.size(), N = s->nodes.size(), Lr = std::max<size_t>(L, 1);
  e.vocab.assign(L, std::map<std::string, int32_t>{{"", 1}});
  e.label_val.assign(Lr * N, 0);
  e.label_num.assign(Lr * N, 0);
  e.label_num_ok.assign(Lr * N, 0);
  for (size_t c = 0; c < L; c++) {
    auto& voc = e.vocab[c];
    const std::string& key = e.label_cols[c];
    for (size_t i = 0; i < N; i++) {
      const Node& n = s->nodes[i];
      std::string v;
      if (key == kObjectName) {
        v = n.name;
      } else {
        auto it = n.labels.find(key);
        if (it == n.labels.end()) continue;
        v = it->second;
      }
      auto vt = voc.find(v);
      int32_t vid;
      if (vt == voc.end()) {
        vid = (int32_t)voc.size() + 1;
        voc[v] = vid;
      } else {
        vid = vt->second;
      }
      e.label_val[c * N + i] = (uint32_t)vid;
      int64_t num;
      if (parse_int64(v, &num)) {
        e.label_num[c * N + i] = num;
        e.label_num_ok[c * N + i] = 1;
      }
    }
  }
}

void build_taints(ksg_snapshot* s) {
  Encoded& e = s->e;
  e.taint_vocab.clear();
  e.taint_id.clear();
  for (auto& n : s->nodes)
    for (auto& t : n.taints)
      if (!e.taint_id.count(t)) {
        e.taint_id[t] = (int)e.taint_vocab.size();
        e.taint_vocab.push_back(t);
      }
  size_t mt = 1;
  for (auto& n : s->nodes) mt = std::max(mt, n.taints.size());
  e.max_taints = (int)mt;
  const size_t N = s->nodes.size();
  e.taints.assign(mt * N, 0);
  for (size_t i = 0; i < N; i++)
    for (size_t k = 0; k < s->nodes[i].taints.size(); k++)
      e.taints[k * N + i] = (uint32_t)e.taint_id[s->nodes[i].taints[k]] + 1;
  e.taint_effect.clear();
  for (auto& t : e.taint_vocab) e.taint_effect.push_back((uint8_t)effect_code(t.effect));
  if (e.taint_effect.empty()) e.taint_effect.push_back(0);
  e.tol_words = std::max<int>(1, ((int)e.taint_vocab.size() + 31) / 32);
  e.taint_strings.clear();
  for (auto& t : e.taint_vocab) e.taint_strings.push_back("{" + t.key + ": " + t.value + "}");
}

// The host-port vocabulary (encoder._build_ports): NodeInfo.UsedPorts only
// ever holds the ports of the snapshot's pods.
void build_ports(ksg_snapshot* s) {
  Encoded& e = s->e;
  std::set<HostPort> all;
  for (auto* lst : {&s->pods, &s->hints})
    for (auto& p : *lst)
      for (auto& hp : pod_host_ports(p)) all.insert(hp);
  e.port_vocab.assign(all.begin(), all.end());
  for (size_t v = 0; v < e.port_vocab.size(); v++) e.port_id[e.port_vocab[v]] = (int)v;
}

void build_images(ksg_snapshot* s) {
  Encoded& e = s->e;
  std::map<std::string, int64_t> first;
  std::map<std::string, std::set<std::string>> with;
  for (auto& n : s->nodes)
    for (auto& img : n.images)
      for (auto& nm : img.names) {
        if (!first.count(nm)) first[nm] = img.size;
        with[nm].insert(n.name);
      }
  e.image_vocab.clear();
  e.image_id.clear();
  e.image_state.clear();
  for (auto& kv : first) {
    e.image_id[kv.first] = (int)e.image_vocab.size();
    e.image_vocab.push_back(kv.first);
    e.image_state[kv.first] = {kv.second, (int64_t)with[kv.first].size()};
  }
  const size_t N = s->nodes.size();
  std::vector<std::vector<uint32_t>> per(N);
  size_t mi = 1;
  for (size_t i = 0; i < N; i++) {
    std::set<int> ids;
    for (auto& img : s->nodes[i].images)
      for (auto& nm : img.names) ids.insert(e.image_id[nm]);
    for (int id : ids) per[i].push_back((uint32_t)id + 1);
    mi = std::max(mi, per[i].size());
  }
  e.max_images = (int)mi;
  e.images.assign(mi * N, 0);
  for (size_t i = 0; i < N; i++)
    for (size_t k = 0; k < per[i].size(); k++) e.images[k * N + i] = per[i][k];
}

// encoder._PodIndex: (key, value) -> pods, to match selectors without a
// pods x selectors scan; returns matching pods in ascending order.
struct PodIndex {
  const std::vector<Pod>& pods;
  std::map<std::pair<std::string, std::string>, std::vector<int>> by_kv;
  explicit PodIndex(const std::vector<Pod>& p) : pods(p) {
    for (size_t i = 0; i < p.size(); i++)
      for (auto& kv : p[i].labels) by_kv[{kv.first, kv.second}].push_back((int)i);
  }
  template <typename Pred>
  std::vector<int> matching(const Canon& canon, Pred pred) const {
    std::vector<int> out;
    if (!canon) return out;
    std::vector<int> tmp, best_store;
    bool have = false;
    for (auto& r : *canon) {
      if (std::get<1>(r) != OP_IN) continue;
      tmp.clear();
      for (auto& v : std::get<2>(r)) {
        auto it = by_kv.find({std::get<0>(r), v});
        if (it != by_kv.end()) tmp.insert(tmp.end(), it->second.begin(), it->second.end());
      }
      if (!have || tmp.size() < best_store.size()) {
        best_store = tmp;
        have = true;
      }
    }
    if (have) {
      std::sort(best_store.begin(), best_store.end());
      best_store.erase(std::unique(best_store.begin(), best_store.end()), best_store.end());
      for (int i : best_store)
        if (pred(pods[i]) && selector_matches(canon, pods[i].labels)) out.push_back(i);
    } else {
      for (size_t i = 0; i < pods.size(); i++)
        if (pred(pods[i]) && selector_matches(canon, pods[i].labels)) out.push_back((int)i);
    }
    return out;
  }
};

void build_topology_universe(ksg_snapshot* s) {
  Encoded& e = s->e;
  const size_t P = s->pods.size();
  e.pts_sel.clear();
  e.pts_order.clear();
  e.ipa_sel.clear();
  e.ipa_order.clear();
  e.templates.clear();
  e.tmpl_order.clear();
  s->owned_templates.assign(P, {});
  for (size_t i = 0; i < P + s->hints.size(); i++) {
    const bool hint = i >= P;
    const Pod& p = hint ? s->hints[i - P] : s->pods[i];
    const PtsPair hint_pts = hint ? pts_constraints(p, s->prof) : PtsPair{};
    const auto& hs = hint ? hint_pts : s->pts_cache[i];
    for (auto* lst : {&hs.first, &hs.second})
      for (auto& c : *lst)
        if (c.canon && !c.canon->empty()) {
          auto key = std::make_pair(*c.canon, p.ns);
          if (!e.pts_sel.count(key)) {
            e.pts_sel[key] = (int)e.pts_order.size();
            e.pts_order.push_back(key);
          }
        }
    auto add_ipa = [&](std::vector<Scope> conj) {
      if (!e.ipa_sel.count(conj)) {
        e.ipa_sel[conj] = (int)e.ipa_order.size();
        e.ipa_order.push_back(conj);
      }
    };
    if (!p.aff_req.empty()) {
      std::vector<Scope> conj;
      for (auto& t : p.aff_req) conj.push_back(term_scope(t, p));
      add_ipa(conj);
    }
    for (auto& t : p.anti_req) add_ipa({term_scope(t, p)});
    for (auto& t : p.aff_pref) add_ipa({term_scope(t, p)});
    for (auto& t : p.anti_pref) add_ipa({term_scope(t, p)});
    auto own = [&](int kind, const AffTerm& t, int wt) {
      auto key = std::make_tuple(kind, term_scope(t, p), e.col_index.at(t.key));
      auto it = e.templates.find(key);
      int tid;
      if (it == e.templates.end()) {
        tid = (int)e.tmpl_order.size();
        e.templates[key] = tid;
        e.tmpl_order.push_back(key);
      } else {
        tid = it->second;
      }
      if (!hint) s->owned_templates[i].emplace_back(tid, wt);
    };
    for (auto& t : p.anti_req) own(TMPL_REQ_ANTI, t, 1);
    for (auto& t : p.aff_req) own(TMPL_REQ_AFF, t, 1);
    for (auto& t : p.aff_pref) own(TMPL_PREF, t, t.weight);
    for (auto& t : p.anti_pref) own(TMPL_PREF, t, -t.weight);
  }
  const int n_pts = (int)e.pts_order.size();
  for (auto& kv : e.ipa_sel) kv.second += n_pts;
  e.n_selectors = n_pts + (int)e.ipa_order.size();
  PodIndex idx(s->pods);
  s->pod_selectors.assign(P, {});
  for (size_t k = 0; k < e.pts_order.size(); k++) {
    const auto& key = e.pts_order[k];
    const std::string& ns = key.second;
    for (int j : idx.matching(Canon(key.first), [&](const Pod& q) { return q.ns == ns && !q.terminating; }))
      s->pod_selectors[j].push_back((int)k);
  }
  for (size_t k = 0; k < e.ipa_order.size(); k++) {
    const auto& conj = e.ipa_order[k];
    std::vector<int> cand;
    bool first = true;
    for (auto& sc : conj) {
      std::vector<int> mt = idx.matching(sc.canon, [&](const Pod& q) { return sc.ns_match(q.ns); });
      if (first) {
        cand = mt;
        first = false;
      } else {
        std::vector<int> inter;
        std::set_intersection(cand.begin(), cand.end(), mt.begin(), mt.end(), std::back_inserter(inter));
        cand = inter;
      }
    }
    for (int j : cand) s->pod_selectors[j].push_back(n_pts + (int)k);
  }
  s->tmpl_match.assign(P, {});
  for (size_t t = 0; t < e.tmpl_order.size(); t++) {
    const int kind = std::get<0>(e.tmpl_order[t]);
    const Scope& sc = std::get<1>(e.tmpl_order[t]);
    for (int j : idx.matching(sc.canon, [&](const Pod& q) { return sc.ns_match(q.ns); }))
      s->tmpl_match[j][kind].push_back((int)t);
  }
  const size_t T = std::max<size_t>(e.tmpl_order.size(), 1);
  e.tmpl_col.assign(T, 0);
  e.tmpl_kind.assign(T, 0);
  e.tmpl_weight.assign(T, 0);
  for (size_t t = 0; t < e.tmpl_order.size(); t++) {
    e.tmpl_col[t] = std::get<2>(e.tmpl_order[t]);
    e.tmpl_kind[t] = std::get<0>(e.tmpl_order[t]);
    e.tmpl_weight[t] = 1;   // unused: per-term weights ride in the owners' commit programs
  }
}

// match_pod's index: every selector (PodTopologySpread), conjunction
// (InterPodAffinity: its first scope) and template of the universe under one
// (key, value) an In requirement of its selector needs, else in the scan list;
// labels.Nothing() matches no pod and is left out.
void build_sel_index(ksg_snapshot* s) {
  Encoded& e = s->e;
  auto& ix = s->sel_index;
  for (int k = 0; k < 3; k++) {
    ix.kv[k].clear();
    ix.scan[k].clear();
  }
  auto put = [&](int which, const std::vector<CReq>& reqs, int id) {
    for (auto& r : reqs)
      if (std::get<1>(r) == OP_IN && !std::get<2>(r).empty()) {
        for (auto& v : std::get<2>(r)) ix.kv[which][{std::get<0>(r), v}].push_back(id);
        return;
      }
    ix.scan[which].push_back(id);
  };
  for (size_t k = 0; k < e.pts_order.size(); k++) put(0, e.pts_order[k].first, (int)k);
  for (size_t k = 0; k < e.ipa_order.size(); k++) {
    const auto& conj = e.ipa_order[k];
    if (conj.empty()) ix.scan[1].push_back((int)k);
    else if (conj[0].canon) put(1, *conj[0].canon, (int)k);
  }
  for (size_t t = 0; t < e.tmpl_order.size(); t++) {
    const Scope& sc = std::get<1>(e.tmpl_order[t]);
    if (sc.canon) put(2, *sc.canon, (int)t);
  }
}

// Selector / template membership of one pod against the current universe
// (the incremental path: the full pass computes it with the pod index): the
// candidates under the pod's (key, value) labels plus the scan lists, each
// checked in full, in id order.
void match_pod(ksg_snapshot* s, int i) {
  Encoded& e = s->e;
  const Pod& q = s->pods[i];
  const auto& ix = s->sel_index;
  auto candidates = [&](int which) {
    std::vector<int> c(ix.scan[which]);
    for (auto& kv : q.labels) {
      auto it = ix.kv[which].find({kv.first, kv.second});
      if (it != ix.kv[which].end()) c.insert(c.end(), it->second.begin(), it->second.end());
    }
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
    return c;
  };
  const int n_pts = (int)e.pts_order.size();
  std::vector<int> sels;
  if (!q.terminating)
    for (int k : candidates(0))
      if (q.ns == e.pts_order[k].second && reqs_match(e.pts_order[k].first, q.labels)) sels.push_back(k);
  for (int k : candidates(1)) {
    bool all = true;
    for (auto& sc : e.ipa_order[k]) all = all && sc.ns_match(q.ns) && selector_matches(sc.canon, q.labels);
    if (all) sels.push_back(n_pts + k);
  }
  s->pod_selectors[i] = sels;
  std::array<std::vector<int>, 3> tm;
  for (int t : candidates(2)) {
    const Scope& sc = std::get<1>(e.tmpl_order[t]);
    if (sc.ns_match(q.ns) && selector_matches(sc.canon, q.labels)) tm[std::get<0>(e.tmpl_order[t])].push_back(t);
  }
  s->tmpl_match[i] = tm;
}

// Universe lookups of an appended pod (no insertion): owned templates,
// PodTopologySpread constraints; sets pass.miss when the pod would extend it.
void prepare_frozen(ksg_snapshot* s, int i, Pass& ps) {
  Encoded& e = s->e;
  const Pod& p = s->pods[i];
  s->req_cache.emplace_back(pod_requests(p, false), pod_requests(p, true));
  for (auto& kv : s->req_cache.back().first)
    if (is_scalar(kv.first) && !e.res_col.count(kv.first)) ps.miss = true;
  s->pts_cache.push_back(pts_constraints(p, s->prof));
  auto& hs = s->pts_cache.back();
  for (auto* lst : {&hs.first, &hs.second})
    for (auto& c : *lst) {
      if (!e.col_index.count(c.key)) ps.miss = true;
      if (c.canon && !c.canon->empty() && !e.pts_sel.count({*c.canon, p.ns})) ps.miss = true;
    }
  auto has_ipa = [&](const std::vector<Scope>& conj) {
    if (!e.ipa_sel.count(conj)) ps.miss = true;
  };
  if (!p.aff_req.empty()) {
    std::vector<Scope> conj;
    for (auto& t : p.aff_req) conj.push_back(term_scope(t, p));
    has_ipa(conj);
  }
  for (auto* v : {&p.anti_req, &p.aff_pref, &p.anti_pref})
    for (auto& t : *v) has_ipa({term_scope(t, p)});
  std::vector<std::pair<int, int>> owned;
  auto own = [&](int kind, const AffTerm& t, int wt) {
    auto ct = e.col_index.find(t.key);
    if (ct == e.col_index.end()) {
      ps.miss = true;
      return;
    }
    auto it = e.templates.find(std::make_tuple(kind, term_scope(t, p), ct->second));
    if (it == e.templates.end()) {
      ps.miss = true;
      return;
    }
    owned.emplace_back(it->second, wt);
  };
  for (auto& hp : pod_host_ports(p))
    if (!e.port_id.count(hp)) ps.miss = true;
  // a pod with claims reads the other pods' claims and the storage objects
  // (shared ReadWriteOncePod / unbound claims): always a full encode
  if (!p.claims.empty()) ps.miss = true;
  for (auto& t : p.anti_req) own(TMPL_REQ_ANTI, t, 1);
  for (auto& t : p.aff_req) own(TMPL_REQ_AFF, t, 1);
  for (auto& t : p.aff_pref) own(TMPL_PREF, t, t.weight);
  for (auto& t : p.anti_pref) own(TMPL_PREF, t, -t.weight);
  if (p.has_node_selector)
    for (auto& kv : p.node_selector)
      if (!e.col_index.count(kv.first)) ps.miss = true;
  auto terms_ok = [&](const Term& t) {
    for (auto& r : t.expr)
      if (!e.col_index.count(r.key)) ps.miss = true;
    if (!t.fields.empty() && !e.col_index.count(kObjectName)) ps.miss = true;
  };
  if (p.has_na_req)
    for (auto& t : p.na_req) terms_ok(t);
  if (p.has_na_pref)
    for (auto& t : p.na_pref) terms_ok(t.pref);
  s->owned_templates.push_back(owned);
  s->pod_selectors.emplace_back();
  s->tmpl_match.emplace_back();
  if (!ps.miss) match_pod(s, i);
}

// ---- per-pod programs --------------------------------------------------------------
// ---- volume plugins ------------------------------------------------------------
// A PreFilter outcome: 1 = rejection (message), 2 = PreFilterResult (names).
struct PreOutcome {
  int kind = 0;
  std::string msg;
  std::set<std::string> names;
};

std::set<std::string> set_and(const std::set<std::string>& a, const std::set<std::string>& b) {
  std::set<std::string> out;
  std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::inserter(out, out.begin()));
  return out;
}

// volumehelpers.LabelZonesToSet: "__"-separated, no blank member
std::vector<std::string> label_zones(const PV& pv, const std::string& value) {
  std::set<std::string> zones;
  size_t at = 0;
  for (;;) {
    const size_t k = value.find("__", at);
    std::string z = value.substr(at, k == std::string::npos ? std::string::npos : k - at);
    const size_t b = z.find_first_not_of(" \t\n\r\f\v"), e = z.find_last_not_of(" \t\n\r\f\v");
    z = b == std::string::npos ? std::string() : z.substr(b, e - b + 1);
    if (z.empty())
      throw EncodeError{KSG_E_UNSUPPORTED, "PersistentVolume " + pv.name + ": zone label '" + value +
                                               "' has an empty member"};
    zones.insert(z);
    if (k == std::string::npos) break;
    at = k + 2;
  }
  return std::vector<std::string>(zones.begin(), zones.end());
}

// encoder.py Encoder._volume_plan [upstream v1.32 volumerestrictions,
// nodevolumelimits/csi.go, volumebinding, volumezone; not vendored: parity
// unpinned, DESIGN.md §9]: the four plugins' PreFilter Skip bits, their
// PreFilter outcomes (into `out`) and the pod's volume program (`words`, the
// grammar of _volume_plan's docstring), value ids taken in the same order.
uint32_t volume_plan(ksg_snapshot* s, int i, const Pod& p, Pass& ps, std::map<int, PreOutcome>& out,
                     std::vector<int32_t>& words, bool& has_words) {
  const uint32_t all_skip = (1u << KSG_PL_VOLUME_RESTRICTIONS) | (1u << KSG_PL_NODE_VOLUME_LIMITS) |
                            (1u << KSG_PL_VOLUME_BINDING) | (1u << KSG_PL_VOLUME_ZONE);
  has_words = false;
  if (p.claims.empty()) return all_skip;
  if (s->csi_limits)
    throw EncodeError{KSG_E_UNSUPPORTED, "pod " + p.ns + "/" + p.name +
                                             ": a node publishes CSI attach limits (NodeVolumeLimits) and the pod "
                                             "has claims"};
  const std::string& ns = p.ns;
  const std::string who = "pod " + ns + "/" + p.name;
  auto claim = [&](const std::string& c) -> const PVC* {
    auto it = s->pvcs.find({ns, c});
    return it == s->pvcs.end() ? nullptr : &it->second;
  };
  auto is_bound = [&](int k) { return s->bound_set.count(k) != 0; };
  auto others_of = [&](const std::string& c) {
    std::set<int> o;
    auto it = s->claim_users.find({ns, c});
    if (it != s->claim_users.end()) o = it->second;
    o.erase(i);
    return o;
  };
  uint32_t skip = 0;
  const std::string* missing = nullptr;
  for (auto& c : p.claims)
    if (!claim(c)) {
      missing = &c;
      break;
    }
  const std::string nf = missing ? "persistentvolumeclaim \"" + *missing + "\" not found" : std::string();
  int32_t flags = 0;
  // VolumeRestrictions: readWriteOncePodPVCsForPod
  if (missing) {
    out[KSG_PL_VOLUME_RESTRICTIONS] = PreOutcome{1, nf, {}};
  } else {
    for (auto& c : p.claims) {
      const PVC* pvc = claim(c);
      if (std::find(pvc->modes.begin(), pvc->modes.end(), "ReadWriteOncePod") == pvc->modes.end()) continue;
      const std::set<int> others = others_of(c);
      if (!is_bound(i))
        for (int u : others)
          if (!is_bound(u))
            throw EncodeError{KSG_E_UNSUPPORTED, who + ": ReadWriteOncePod claim '" + c +
                                                     "' is shared with another queued pod (whose placement decides "
                                                     "the conflict)"};
      if (!others.empty()) flags |= kVolRwopConflict;   // StorageInfos.IsPVCUsedByPods
    }
  }
  // VolumeBinding: podHasPVCs, GetPodVolumeClaims, GetEligibleNodes
  std::vector<const PVC*> bound;
  std::vector<std::pair<const PVC*, const SClass*>> prov;
  bool vb_set = false;
  PreOutcome vb;
  for (auto& c : p.claims) {
    const PVC* pvc = claim(c);
    if (!pvc) {
      vb = PreOutcome{1, nf, {}};
      vb_set = true;
      break;
    }
    if (pvc->deleting) {
      vb = PreOutcome{1, "persistentvolumeclaim \"" + c + "\" is being deleted", {}};
      vb_set = true;
      break;
    }
  }
  if (!vb_set) {
    bool immediate = false;
    for (auto& c : p.claims) {
      const PVC* pvc = claim(c);
      if (pvc->fully_bound()) {
        bound.push_back(pvc);
        continue;
      }
      auto ct = pvc->storage_class.empty() ? s->classes.end() : s->classes.find(pvc->storage_class);
      if (ct != s->classes.end() && ct->second.mode == kWFFC && pvc->volume_name.empty())
        prov.emplace_back(pvc, &ct->second);
      else
        immediate = true;
    }
    if (immediate) {
      vb = PreOutcome{1, "pod has unbound immediate PersistentVolumeClaims", {}};
      vb_set = true;
    }
  }
  if (!vb_set) {
    std::optional<std::set<std::string>> eligible;
    for (const PVC* pvc : bound) {   // util.GetLocalPersistentVolumeNodeNames of every bound PV
      auto pt = s->pvs.find(pvc->volume_name);
      if (pt == s->pvs.end()) {
        eligible.reset();
        break;
      }
      std::set<std::string> names;
      if (pt->second.has_na)
        for (auto& t : pt->second.na) {
          std::optional<std::set<std::string>> tn;
          for (auto& r : t.expr)
            if (r.key == kHostname && r.op == "In") {
              std::set<std::string> sv(r.values.begin(), r.values.end());
              tn = tn ? set_and(*tn, sv) : sv;
            }
          if (tn) names.insert(tn->begin(), tn->end());
        }
      if (!names.empty()) eligible = eligible ? set_and(*eligible, names) : names;
    }
    if (eligible) {
      vb = PreOutcome{2, "", *eligible};
      vb_set = true;
    }
    for (auto& pr : prov) {
      for (auto& kv : s->pvs) {
        const PV& pv = kv.second;
        if (pv.storage_class == pr.first->storage_class &&
            (!pv.has_claim_ref || (pv.claim_ns == ns && pv.claim_name == pr.first->name)))
          throw EncodeError{KSG_E_UNSUPPORTED, who + ": claim '" + pr.first->name +
                                                   "' could bind statically to PersistentVolume '" + pv.name +
                                                   "' (findMatchingVolumes is not modelled)"};
      }
      if (!is_bound(i) && !others_of(pr.first->name).empty())
        throw EncodeError{KSG_E_UNSUPPORTED, who + ": unbound claim '" + pr.first->name +
                                                 "' is shared with another pod (its assumed binding is not modelled)"};
    }
  }
  if (vb_set) out[KSG_PL_VOLUME_BINDING] = vb;
  // VolumeZone: getPVbyPod
  std::vector<std::pair<std::string, std::vector<std::string>>> zone;
  bool vz_set = false;
  std::string vz;
  for (auto& c : p.claims) {
    if (c.empty()) {
      vz = "PersistentVolumeClaim had no name";
      vz_set = true;
      break;
    }
    const PVC* pvc = claim(c);
    if (!pvc) {
      vz = "persistentvolumeclaim \"" + c + "\" not found";
      vz_set = true;
      break;
    }
    if (pvc->volume_name.empty()) {
      const std::string& sc = pvc->storage_class;
      if (sc.empty()) {
        vz = "PersistentVolumeClaim had no pv name and storageClass name";
        vz_set = true;
        break;
      }
      auto ct = s->classes.find(sc);
      if (ct == s->classes.end()) {
        vz = "storageclass.storage.k8s.io \"" + sc + "\" not found";
        vz_set = true;
        break;
      }
      if (ct->second.mode == kWFFC) continue;
      vz = "PersistentVolume had no name";
      vz_set = true;
      break;
    }
    auto pt = s->pvs.find(pvc->volume_name);
    if (pt == s->pvs.end()) {
      vz = "persistentvolume \"" + pvc->volume_name + "\" not found";
      vz_set = true;
      break;
    }
    for (const char* key : kZoneLabels) {
      auto lt = pt->second.labels.find(key);
      if (lt != pt->second.labels.end()) zone.emplace_back(key, label_zones(pt->second, lt->second));
    }
  }
  if (vz_set)
    out[KSG_PL_VOLUME_ZONE] = PreOutcome{1, vz, {}};
  else if (zone.empty())
    skip |= 1u << KSG_PL_VOLUME_ZONE;
  // the Filter program
  words = {flags, (int32_t)bound.size()};
  static const char* const kMigrated[] = {"gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "azureFile",
                                          "cinder", "vsphereVolume", "portworxVolume"};
  for (const PVC* pvc : bound) {
    auto pt = s->pvs.find(pvc->volume_name);
    if (pt == s->pvs.end()) {
      words.push_back(0);
      continue;
    }
    const PV& pv = pt->second;
    for (const char* m : kMigrated)
      if (pv.source == m)
        throw EncodeError{KSG_E_UNSUPPORTED, "PersistentVolume " + pv.name + ": " + pv.source +
                                                 " (CSI translation not modelled)"};
    if (!pv.has_na) {
      words.insert(words.end(), {1, -1});
      continue;
    }
    std::vector<std::vector<int32_t>> terms;
    bool nameless = false;   // a fields-only term: CheckNodeAffinity's nameless node matches it
    for (auto& t : pv.na) {
      if (t.expr.empty()) {
        if (!t.fields.empty()) {
          nameless = true;
          break;
        }
        terms.push_back({0});   // an empty term matches nothing
        continue;
      }
      std::vector<int32_t> tw = {(int32_t)t.expr.size()};
      for (auto& r : t.expr) ps.emit(tw, ps.requirement(r, false));
      terms.push_back(std::move(tw));
    }
    if (nameless) {
      words.insert(words.end(), {1, -1});
    } else {
      words.insert(words.end(), {1, (int32_t)terms.size()});
      for (auto& tw : terms) ps.emit(words, tw);
    }
  }
  words.push_back((int32_t)prov.size());
  for (auto& pr : prov) {
    auto at = pr.first->ann.find("volume.kubernetes.io/selected-node");
    int32_t sel = -1;
    if (at != pr.first->ann.end()) {
      auto nt = s->node_index.find(at->second);
      sel = nt == s->node_index.end() ? -2 : nt->second;
    }
    const SClass& cls = *pr.second;
    if (cls.provisioner.empty() || cls.provisioner == "kubernetes.io/no-provisioner") {
      words.insert(words.end(), {sel, -1});
      continue;
    }
    words.insert(words.end(), {sel, (int32_t)cls.topo.size()});
    for (auto& term : cls.topo) {
      words.push_back((int32_t)term.size());
      for (auto& kv : term) {
        const int col = ps.col(kv.first);
        std::set<int32_t> ids;
        for (auto& v : kv.second) ids.insert(ps.value_id(col, v));
        if (ids.empty()) {
          words.insert(words.end(), {0, OP_NEVER, 0});
        } else {
          words.insert(words.end(), {col, OP_IN, (int32_t)ids.size()});
          words.insert(words.end(), ids.begin(), ids.end());
        }
      }
    }
  }
  for (const char* k : kZoneLabels) {
    auto it = s->e.col_index.find(k);
    words.push_back(it == s->e.col_index.end() ? -1 : it->second);
  }
  words.push_back((int32_t)zone.size());
  for (auto& kv : zone) {
    const int col = ps.col(kv.first), gcol = ps.col(ga_label(kv.first));
    std::set<int32_t> ids, gids;
    for (auto& v : kv.second) ids.insert(ps.value_id(col, v));
    for (auto& v : kv.second) gids.insert(ps.value_id(gcol, v));
    words.insert(words.end(), {col, gcol, (int32_t)ids.size()});
    words.insert(words.end(), ids.begin(), ids.end());
    words.push_back((int32_t)gids.size());
    words.insert(words.end(), gids.begin(), gids.end());
  }
  has_words = true;
  return skip;
}

void encode_pod(ksg_snapshot* s, int i, Pass& ps) {
  Encoded& e = s->e;
  const Pod& p = s->pods[i];
  const Profile& prof = s->prof;
  std::vector<int32_t>& prog = e.prog;
  const ResMap& r = s->req_cache[i].first;
  const ResMap& nz = s->req_cache[i].second;
  ksg_pod rec;
  std::memset(&rec, 0, sizeof(rec));
  for (auto& kv : r) {
    auto it = e.res_col.find(kv.first);
    if (it != e.res_col.end()) rec.req[it->second] = kv.second;
  }
  auto get = [](const ResMap& m, const std::string& k) {
    auto it = m.find(k);
    return it == m.end() ? (int64_t)0 : it->second;
  };
  rec.nz_cpu = get(nz, kCPU);
  rec.nz_mem = get(nz, kMemory);
  uint32_t flags = 0;
  const Taint unsched{kUnschedTaint, "", "NoSchedule"};
  for (auto& t : p.tols)
    if (t.tolerates(unsched)) {
      flags |= KSG_POD_TOL_UNSCHED;
      break;
    }
  const bool na_required = p.has_node_selector || p.has_na_req;
  if (na_required) flags |= KSG_POD_NA_REQUIRED;
  bool best_effort = true;
  for (auto& br : prof.ba_res)
    if (e.res_col.count(br.first) && get(r, br.first) != 0) best_effort = false;
  if (best_effort) flags |= KSG_POD_BEST_EFFORT;
  uint32_t fskip = 0, sskip = 0;
  if (!na_required) fskip |= 1u << KSG_PL_NODE_AFFINITY;
  const std::vector<HostPort> hports = pod_host_ports(p);
  if (hports.empty()) fskip |= 1u << KSG_PL_NODE_PORTS;   // nodeports PreFilter: Skip without ports
  // the volume plugins' PreFilter (Skip for a pod without claims) and program
  std::map<int, PreOutcome> outcome;
  std::vector<int32_t> vol_words;
  bool has_vol = false;
  if (s->vol_run) {
    fskip |= volume_plan(s, i, p, ps, outcome, vol_words, has_vol);
  } else {
    for (int v : {KSG_PL_VOLUME_RESTRICTIONS, KSG_PL_NODE_VOLUME_LIMITS, KSG_PL_VOLUME_BINDING, KSG_PL_VOLUME_ZONE})
      fskip |= 1u << v;
  }
  const auto& hard = s->pts_cache[i].first;
  const auto& soft = s->pts_cache[i].second;
  if (hard.empty()) fskip |= 1u << KSG_PL_POD_TOPOLOGY_SPREAD;
  if (soft.empty()) sskip |= 1u << KSG_PL_POD_TOPOLOGY_SPREAD;
  if (!p.has_na_pref) sskip |= 1u << KSG_PL_NODE_AFFINITY;
  sskip |= 1u << KSG_PL_VOLUME_BINDING;
  if (prof.ba_skip_be && (flags & KSG_POD_BEST_EFFORT)) sskip |= 1u << KSG_PL_BALANCED_ALLOCATION;
  const bool pref_pod_aff = !p.aff_pref.empty() || !p.anti_pref.empty();
  if (prof.ignore_pref && !pref_pod_aff) sskip |= 1u << KSG_PL_INTER_POD_AFFINITY;
  // NodeAffinity PreFilter: matchFields metadata.name In -> PreFilterResult
  if (p.has_na_req && !p.na_req.empty()) {
    std::optional<std::set<std::string>> names_u;
    bool all_named = true;
    for (auto& term : p.na_req) {
      std::optional<std::set<std::string>> tn;
      for (auto& rq : term.fields)
        if (rq.key == kObjectName && rq.op == "In") {
          std::set<std::string> sv(rq.values.begin(), rq.values.end());
          tn = tn ? set_and(*tn, sv) : sv;
        }
      if (!tn) {
        all_named = false;
        break;
      }
      if (!names_u) names_u = *tn;
      else names_u->insert(tn->begin(), tn->end());
    }
    if (all_named && names_u)
      outcome[KSG_PL_NODE_AFFINITY] = names_u->empty() ? PreOutcome{1, "pod affinity terms conflict", {}}
                                                        : PreOutcome{2, "", *names_u};
  }
  // PreFilter outcomes in the profile's PreFilter order (RunPreFilterPlugins):
  // the first rejection ends the cycle; PreFilterResults merge by
  // intersection, and an empty merge ends it too (the framework's message)
  rec.node_set = -1;
  e.prefilter_names.erase(i);
  e.prefilter_reject.erase(i);
  std::optional<std::set<std::string>> merged;
  for (int pid : prof.order[KSG_POINT_PREFILTER]) {
    auto it = outcome.find(pid);
    if (it == outcome.end()) continue;
    const PreOutcome& o = it->second;
    if (o.kind == 1) {
      flags |= KSG_POD_PREFILTER_REJECT;
      e.prefilter_reject[i] = {pid, o.msg};
      break;
    }
    if (o.kind == 2) {
      e.prefilter_names[i][pid] = std::vector<std::string>(o.names.begin(), o.names.end());
      merged = merged ? set_and(*merged, o.names) : o.names;
      if (merged->empty()) {
        flags |= KSG_POD_PREFILTER_REJECT;
        e.prefilter_reject[i] = {pid, std::string()};
        break;
      }
    }
  }
  if (merged && !merged->empty() && !(flags & KSG_POD_PREFILTER_REJECT)) {
    const int N = (int)s->nodes.size(), W = (N + 31) / 32;
    std::vector<uint32_t> bits(W, 0);
    for (auto& nm : *merged) {
      auto it = s->node_index.find(nm);
      if (it != s->node_index.end()) bits[it->second / 32] |= 1u << (it->second % 32);
    }
    rec.node_set = (int32_t)prog.size();
    for (uint32_t b : bits) prog.push_back((int32_t)b);
  }
  rec.flags = flags;
  rec.filter_skip = fskip;
  rec.score_skip = sskip;
  if (p.node_name.empty()) {
    rec.node_name = -1;
  } else {
    auto it = s->node_index.find(p.node_name);
    rec.node_name = it == s->node_index.end() ? -2 : it->second;
  }
  rec.n_containers = (int32_t)(p.containers.size() + p.init.size());
  const int32_t blob = (int32_t)prog.size();
  // tol := filter_bits[W] prefer_bits[W]
  {
    const int W = e.tol_words;
    std::vector<uint32_t> fb(W, 0), pb(W, 0);
    std::vector<const Tol*> pref;
    for (auto& t : p.tols)
      if (t.effect.empty() || t.effect == "PreferNoSchedule") pref.push_back(&t);
    for (size_t v = 0; v < e.taint_vocab.size(); v++) {
      const Taint& taint = e.taint_vocab[v];
      bool f = false, pr = false;
      for (auto& t : p.tols) f = f || t.tolerates(taint);
      for (auto* t : pref) pr = pr || t->tolerates(taint);
      if (f) fb[v / 32] |= 1u << (v % 32);
      if (pr) pb[v / 32] |= 1u << (v % 32);
    }
    rec.tol = (int32_t)prog.size();
    for (uint32_t x : fb) prog.push_back((int32_t)x);
    for (uint32_t x : pb) prog.push_back((int32_t)x);
  }
  // na_req := n_sel requirement[n_sel] n_terms { n_reqs requirement[n_reqs] }
  rec.na_req = -1;
  if (na_required) {
    std::vector<int32_t> w;
    w.push_back((int32_t)p.node_selector.size());
    for (auto& kv : p.node_selector) {   // std::map: sorted by key
      const int c = ps.col(kv.first);
      const int32_t id = ps.miss ? 0 : ps.value_id(c, kv.second);
      w.insert(w.end(), {c, OP_IN, 1, id});
    }
    if (!p.has_na_req) {
      w.push_back(-1);
    } else {
      w.push_back((int32_t)p.na_req.size());
      for (auto& t : p.na_req) ps.emit(w, ps.term(t));
    }
    rec.na_req = (int32_t)prog.size();
    ps.emit(prog, w);
  }
  // na_pref := n_terms { weight n_reqs requirement[n_reqs] }
  rec.na_pref = -1;
  if (p.has_na_pref) {
    std::vector<int32_t> w = {0};
    for (auto& pt : p.na_pref) {
      if (pt.weight == 0 || (pt.pref.expr.empty() && pt.pref.fields.empty())) continue;
      w[0]++;
      w.push_back(pt.weight);
      ps.emit(w, ps.term(pt.pref));
    }
    rec.na_pref = (int32_t)prog.size();
    ps.emit(prog, w);
  }
  // img := n { image_id+1 contrib_lo contrib_hi }
  {
    std::vector<int32_t> ents;
    const double total = (double)s->nodes.size();
    auto one = [&](const Container& c) {
      const std::string nm = normalized_image(c.image);
      auto it = e.image_state.find(nm);
      if (it == e.image_state.end()) return;
      const int64_t contrib = (int64_t)((double)it->second.first * ((double)it->second.second / total));
      const uint64_t u = (uint64_t)contrib;
      ents.insert(ents.end(), {e.image_id[nm] + 1, s32(u), s32(u >> 32)});
    };
    for (auto& c : p.init) one(c);
    for (auto& c : p.containers) one(c);
    rec.img = (int32_t)prog.size();
    prog.push_back((int32_t)(ents.size() / 3));
    ps.emit(prog, ents);
  }
  // pts := n_hard n_soft require_all {hard}[..] {soft}[..]
  rec.pts = -1;
  if (!hard.empty() || !soft.empty()) {
    const int require_all = (!p.spread.empty() || !prof.pts_system) ? 1 : 0;
    std::vector<int32_t> w = {(int32_t)hard.size(), (int32_t)soft.size(), require_all};
    auto sel_of = [&](const Canon& c) -> int32_t {
      if (!c || c->empty()) return -1;
      auto it = e.pts_sel.find({*c, p.ns});
      if (it == e.pts_sel.end()) {
        ps.miss = true;
        return -1;
      }
      return it->second;
    };
    for (auto& c : hard) {
      const int self = (c.canon && selector_matches(c.canon, p.labels)) ? 1 : 0;
      w.insert(w.end(), {ps.col(c.key), sel_of(c.canon), c.skew, c.min_domains, self, c.na_honor ? 1 : 0,
                         c.nt_honor ? 1 : 0});
    }
    for (auto& c : soft)
      w.insert(w.end(), {ps.col(c.key), sel_of(c.canon), c.skew, c.na_honor ? 1 : 0, c.nt_honor ? 1 : 0,
                         c.key == kHostname ? 1 : 0});
    rec.pts = (int32_t)prog.size();
    ps.emit(prog, w);
  }
  // ipa
  rec.ipa = -1;
  {
    const auto& tm = s->tmpl_match[i];
    const bool any = !p.aff_req.empty() || !p.anti_req.empty() || !p.aff_pref.empty() || !p.anti_pref.empty() ||
                     !tm[0].empty() || !tm[1].empty() || !tm[2].empty();
    if (any) {
      std::vector<int32_t> w;
      auto sel_id = [&](const std::vector<Scope>& conj) -> int32_t {
        auto it = e.ipa_sel.find(conj);
        if (it == e.ipa_sel.end()) {
          ps.miss = true;
          return -1;
        }
        return it->second;
      };
      if (!p.aff_req.empty()) {
        std::vector<Scope> scopes;
        for (auto& t : p.aff_req) scopes.push_back(term_scope(t, p));
        bool self_all = true;
        for (auto& sc : scopes) self_all = self_all && sc.ns_match(p.ns) && selector_matches(sc.canon, p.labels);
        w.insert(w.end(), {(int32_t)p.aff_req.size(), sel_id(scopes), self_all ? 1 : 0});
        for (auto& t : p.aff_req) w.push_back(ps.col(t.key));
      } else {
        w.insert(w.end(), {0, -1, 0});
      }
      w.push_back((int32_t)p.anti_req.size());
      for (auto& t : p.anti_req) w.insert(w.end(), {ps.col(t.key), sel_id({term_scope(t, p)})});
      w.push_back((int32_t)(p.aff_pref.size() + p.anti_pref.size()));
      for (auto& t : p.aff_pref) w.insert(w.end(), {ps.col(t.key), sel_id({term_scope(t, p)}), t.weight});
      for (auto& t : p.anti_pref) w.insert(w.end(), {ps.col(t.key), sel_id({term_scope(t, p)}), -t.weight});
      for (int k = 0; k < 3; k++) {
        w.push_back((int32_t)tm[k].size());
        w.insert(w.end(), tm[k].begin(), tm[k].end());
      }
      rec.ipa = (int32_t)prog.size();
      ps.emit(prog, w);
    }
  }
  // commit := n_sel sel[n_sel] n_tmpl {tmpl weight}[n_tmpl]
  rec.commit = -1;
  {
    std::vector<int> sels = s->pod_selectors[i];
    std::sort(sels.begin(), sels.end());
    const auto& tmo = s->owned_templates[i];
    if (!sels.empty() || !tmo.empty()) {
      rec.commit = (int32_t)prog.size();
      prog.push_back((int32_t)sels.size());
      prog.insert(prog.end(), sels.begin(), sels.end());
      prog.push_back((int32_t)tmo.size());
      for (auto& pr : tmo) prog.insert(prog.end(), {pr.first, pr.second});
    }
  }
  // ports := n_conf conf[n_conf] n_own own[n_own] (HostPortInfo.CheckConflict
  // over the vocabulary; own = what the pod's assume adds to UsedPorts)
  rec.ports = -1;
  rec.vol = -1;
  rec.pad = 0;
  if (!hports.empty()) {
    std::set<int32_t> conf, own;
    for (auto& hp : hports) {
      auto it = e.port_id.find(hp);
      if (it == e.port_id.end()) {   // frozen pass: the vocabulary would grow
        ps.miss = true;
        break;
      }
      own.insert(it->second);
      const std::string& ip = std::get<0>(hp);
      for (size_t v = 0; v < e.port_vocab.size(); v++) {
        const HostPort& q = e.port_vocab[v];
        if (std::get<1>(q) == std::get<1>(hp) && std::get<2>(q) == std::get<2>(hp) &&
            (ip == kBindAllHostIP || std::get<0>(q) == kBindAllHostIP || std::get<0>(q) == ip))
          conf.insert((int32_t)v);
      }
    }
    rec.ports = (int32_t)prog.size();
    prog.push_back((int32_t)conf.size());
    prog.insert(prog.end(), conf.begin(), conf.end());
    prog.push_back((int32_t)own.size());
    prog.insert(prog.end(), own.begin(), own.end());
  }
  if (has_vol) {
    rec.vol = (int32_t)prog.size();
    ps.emit(prog, vol_words);
  }
  rec.blob = blob;
  rec.blob_len = (int32_t)prog.size() - blob;
  if ((int)e.pods.size() <= i) e.pods.resize(i + 1);
  e.pods[i] = rec;
}

// Requirement values may extend a column's vocabulary after the node columns
// were built; ids stay below col_vocab either way.
void finish_arrays(ksg_snapshot* s) {
  Encoded& e = s->e;
  e.col_vocab.clear();
  for (auto& v : e.vocab) e.col_vocab.push_back((int32_t)v.size() + 1);
  if (e.col_vocab.empty()) e.col_vocab.push_back(1);
}

void encode_all(ksg_snapshot* s) {
  Encoded& e = s->e;
  e = Encoded{};
  const size_t N = s->nodes.size(), P = s->pods.size();
  e.N = (int)N;
  build_resources(s);
  build_label_columns(s);
  build_taints(s);
  build_images(s);
  build_ports(s);
  build_topology_universe(s);
  build_sel_index(s);
  // node columns
  const size_t R = e.res_names.size();
  e.alloc.assign(R * N, 0);
  for (size_t i = 0; i < N; i++)
    for (auto& kv : s->nodes[i].alloc) {
      auto it = e.res_col.find(kv.first);
      if (it != e.res_col.end()) e.alloc[(size_t)it->second * N + i] = kv.second;
    }
  e.requested.assign(R * N, 0);
  e.nonzero.assign(2 * N, 0);
  e.allowed.assign(N, 0);
  e.pod_count.assign(N, 0);
  e.unsched.assign(N, 0);
  for (size_t i = 0; i < N; i++) {
    auto it = s->nodes[i].alloc.find(kPods);
    e.allowed[i] = it == s->nodes[i].alloc.end() ? 0 : (int32_t)it->second;
    e.unsched[i] = s->nodes[i].unsched ? 1 : 0;
  }
  const size_t Lc = e.label_cols.size();
  e.col_unique.assign(std::max<size_t>(Lc, 1), 0);
  for (size_t c = 0; c < Lc; c++) {
    std::set<uint32_t> seen;
    bool uniq = true;
    for (size_t i = 0; i < N && uniq; i++) {
      const uint32_t v = e.label_val[c * N + i];
      if (v && !seen.insert(v).second) uniq = false;
    }
    e.col_unique[c] = uniq ? 1 : 0;
  }
  e.log_table.resize(N + 3);
  for (size_t i = 0; i < N + 3; i++) e.log_table[i] = go_log((double)i);
  // pods: the volume plugins' view of the other pods (claim users, bindings)
  s->claim_users.clear();
  for (size_t i = 0; i < P; i++)
    for (auto& c : s->pods[i].claims) s->claim_users[{s->pods[i].ns, c}].insert((int)i);
  s->bound_set.clear();
  for (auto& b : s->binds) s->bound_set.insert(b.first);
  s->vol_run = false;
  bool nvl = false;
  for (int pt : {KSG_POINT_PREFILTER, KSG_POINT_FILTER})
    for (int pid : s->prof.order[pt]) {
      s->vol_run = s->vol_run || pid == KSG_PL_VOLUME_RESTRICTIONS || pid == KSG_PL_NODE_VOLUME_LIMITS ||
                   pid == KSG_PL_VOLUME_BINDING || pid == KSG_PL_VOLUME_ZONE;
      nvl = nvl || pid == KSG_PL_NODE_VOLUME_LIMITS;
    }
  s->csi_limits = false;
  for (auto& n : s->nodes)
    for (auto& kv : n.alloc) s->csi_limits = s->csi_limits || (nvl && starts_with(kv.first, "attachable-volumes-csi-"));
  e.pods.assign(P, ksg_pod{});
  Pass ps{s, false};
  for (size_t i = 0; i < P; i++) encode_pod(s, (int)i, ps);
  finish_arrays(s);
  s->encoded = true;
  s->n_encoded = (int)P;
  s->hints_seen = s->hints.size();
  s->epoch++;
}

// ---- profile ---------------------------------------------------------------------
std::string plain_name(std::string n) {
  if (n.size() > 7 && n.compare(n.size() - 7, 7, "Wrapped") == 0) n.resize(n.size() - 7);
  return n;
}
int plugin_id(const std::string& plain) {
  for (int k = 0; k < KSG_NPLUGINS; k++)
    if (plain == kPluginNames[k]) return k;
  return -1;
}
bool non_eval(const std::string& plain) {
  for (const char* n : kNonEval)
    if (plain == n) return true;
  return false;
}

// The framework's plugin list of extension point `pt` (extension index ext):
// profile.py Profile._expand [upstream v1.32 expandMultiPointPlugins, TO
// VERIFY, DESIGN.md §9].  Returns false with a message for a configuration
// the framework (or the simulator's registry, plugins.go:39-60) refuses.
bool expand_point(const ksg_plugin_set_view& ps, const std::vector<int>& enabled, int ext, std::vector<int>& out,
                  std::string& err) {
  std::vector<int> multi;
  for (int pid : enabled)
    if (kExt[pid][ext]) multi.push_back(pid);
  if (ps.n_enabled <= 0 && ps.n_disabled <= 0) {
    out = multi;
    return true;
  }
  std::vector<int> own;
  for (int32_t i = 0; i < ps.n_enabled; i++) {
    const std::string n = plain_name(S(ps.enabled[i].name));
    const int pid = plugin_id(n);
    if (pid < 0) {
      err = "plugin " + n + " is not an in-tree Filter/Score plugin";
      return false;
    }
    if (!kExt[pid][ext]) {
      err = "plugin " + n + " does not extend this point";
      return false;
    }
    if (std::find(own.begin(), own.end(), pid) != own.end()) {
      err = "plugin " + n + " listed twice";
      return false;
    }
    own.push_back(pid);
  }
  bool all = false;
  std::set<int> off;
  for (int32_t i = 0; i < ps.n_disabled; i++) {
    const std::string n = S(ps.disabled[i]);
    if (n == "*") all = true;
    const int pid = plugin_id(plain_name(n));
    if (pid >= 0) off.insert(pid);
  }
  out.clear();
  if (all) {
    out = own;
    return true;
  }
  auto in = [](const std::vector<int>& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); };
  for (int pid : own)
    if (in(multi, pid)) out.push_back(pid);
  for (int pid : multi)
    if (!off.count(pid) && !in(own, pid)) out.push_back(pid);
  for (int pid : own)
    if (!in(multi, pid)) out.push_back(pid);
  return true;
}

// Orders of the four modelled points and the two weight maps.
bool derive_profile(Profile& p, const ksg_profile_view* pv, std::string& err) {
  static const int kExtOf[KSG_NPOINTS] = {0, 1, 2, 3};   // prefilter, filter, prescore, score
  for (int pt = 0; pt < KSG_NPOINTS; pt++)
    if (!expand_point(pv->points[pt], p.enabled, kExtOf[pt], p.order[pt], err)) return false;
  // Score.Enabled then MultiPoint.Enabled (plugins.go:291-292)
  std::vector<std::pair<std::string, int32_t>> seq;
  const ksg_plugin_set_view& sc = pv->points[KSG_POINT_SCORE];
  for (int32_t i = 0; i < sc.n_enabled; i++) seq.emplace_back(S(sc.enabled[i].name), sc.enabled[i].weight);
  seq.insert(seq.end(), p.plugins.begin(), p.plugins.end());
  for (auto& kv : seq) {
    const int pid = plugin_id(plain_name(kv.first));
    if (pid < 0) continue;
    const int32_t w = kv.second != 0 ? kv.second : 1;
    p.store_w[pid] = w;                   // the store map: a later entry replaces (plugins.go:293-301)
    if (p.sel_w[pid] == 0) p.sel_w[pid] = w;   // the framework: the point's own weight first
  }
  return true;
}

int encode_profile(ksg_snapshot* s) {
  const Profile& pr = s->prof;
  Encoded& e = s->e;
  ksg_profile& p = e.prof;
  std::memset(&p, 0, sizeof(p));
  for (int pid : pr.order[KSG_POINT_FILTER]) p.filter_order[p.n_filter++] = pid;
  for (int pid : pr.order[KSG_POINT_SCORE]) {
    p.score_mask |= 1u << pid;
    p.weight[pid] = pr.sel_w[pid] != 0 ? pr.sel_w[pid] : 1;
  }
  p.fit_strategy = pr.fit_strategy == "MostAllocated"              ? KSG_MOST_ALLOCATED
                   : pr.fit_strategy == "RequestedToCapacityRatio" ? KSG_REQUESTED_TO_CAPACITY_RATIO
                                                                   : KSG_LEAST_ALLOCATED;
  if (p.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO)
    for (auto& pt : pr.shape) {   // scores scaled by MaxNodeScore / MaxCustomPriorityScore
      p.shape_util[p.shape_n] = pt.first;
      p.shape_score[p.shape_n++] = pt.second * 10;
    }
  for (auto& r : pr.fit_res) {
    auto it = e.res_col.find(r.first);
    if (it == e.res_col.end()) continue;
    p.fit_res[p.fit_n] = it->second;
    p.fit_w[p.fit_n] = r.second;
    p.fit_n++;
  }
  for (auto& r : pr.ba_res) {
    auto it = e.res_col.find(r.first);
    if (it != e.res_col.end()) p.ba_res[p.ba_n++] = it->second;
  }
  for (size_t c = 0; c < e.res_names.size(); c++) {
    const std::string& r = e.res_names[c];
    const auto slash = r.find('/');
    if (slash == std::string::npos) continue;
    if (pr.ignored.count(r) || pr.ignored_groups.count(r.substr(0, slash))) p.fit_ignored_res |= 1u << c;
  }
  p.hard_pod_affinity_weight = pr.hard_weight;
  p.flags = (pr.ba_skip_be ? KSG_PROF_BA_SKIP_BEST_EFFORT : 0u) | (pr.ignore_pref ? KSG_PROF_IPA_IGNORE_EXISTING_PREF : 0u);
  return KSG_OK;
}

int do_encode(ksg_snapshot* s) {
  try {
    encode_all(s);
    encode_profile(s);
  } catch (const EncodeError& x) {
    s->encoded = false;
    return fail(s, x.code, x.msg);
  } catch (const std::exception& x) {
    s->encoded = false;
    return fail(s, KSG_E_INVALID, std::string("encode: ") + x.what());
  }
  return KSG_OK;
}

void fill_views(ksg_snapshot* s, ksg_nodes* nd, ksg_topology* tp, ksg_workload* wl, ksg_profile* pf) {
  Encoded& e = s->e;
  if (nd) {
    *nd = ksg_nodes{};
    nd->n_nodes = e.N;
    nd->n_res = (int32_t)e.res_names.size();
    nd->alloc = e.alloc.data();
    nd->requested = e.requested.data();
    nd->nonzero = e.nonzero.data();
    nd->allowed_pods = e.allowed.data();
    nd->pod_count = e.pod_count.data();
    nd->unschedulable = e.unsched.data();
    nd->n_label_cols = (int32_t)e.label_cols.size();
    nd->label_val = e.label_val.data();
    nd->label_num = e.label_num.data();
    nd->label_num_ok = e.label_num_ok.data();
    nd->max_taints = e.max_taints;
    nd->taints = e.taints.data();
    nd->n_taint_vocab = (int32_t)e.taint_vocab.size();
    nd->taint_effect = e.taint_effect.data();
    nd->max_images = e.max_images;
    nd->images = e.images.data();
    nd->n_images = (int32_t)e.image_vocab.size();
    nd->n_port_vocab = (int32_t)e.port_vocab.size();
  }
  if (tp) {
    *tp = ksg_topology{};
    tp->n_selectors = e.n_selectors;
    tp->n_templates = (int32_t)e.tmpl_order.size();
    tp->tmpl_col = e.tmpl_col.data();
    tp->tmpl_kind = e.tmpl_kind.data();
    tp->tmpl_weight = e.tmpl_weight.data();
    tp->col_vocab = e.col_vocab.data();
    tp->col_unique = e.col_unique.data();
    tp->log_table = e.log_table.data();
    tp->log_n = (int32_t)e.log_table.size();
  }
  if (wl) {
    *wl = ksg_workload{};
    wl->pods = e.pods.data();
    wl->n_pods = (int32_t)e.pods.size();
    static const int32_t kEmpty[1] = {0};   // encoder.py: `prog or [0]`
    wl->prog = e.prog.empty() ? kEmpty : e.prog.data();
    wl->prog_len = std::max<int64_t>((int64_t)e.prog.size(), 1);
  }
  if (pf) *pf = e.prof;
}

// Encode the pods added since the last encode.  When none of them extends
// the encoding universe (label columns, value ids, resource columns,
// selectors, term templates) they are encoded against it and appended
// (*appended = 1): byte-identical to a full re-encode, which is what runs
// otherwise (*appended = 0).
// Whether pod p (a hint) would extend the encoding universe: it is encoded
// against the frozen universe at index P, exactly as an append would, and
// everything that touched is undone.  Needs every pod encoded (caches sized P).
bool extends_universe(ksg_snapshot* s, const Pod& p) {
  Encoded& e = s->e;
  const int P = (int)s->pods.size();
  const size_t prog0 = e.prog.size(), pods0 = e.pods.size(), caches0 = s->req_cache.size();
  s->pods.push_back(p);
  bool miss = false;
  try {
    Pass ps{s, true};
    prepare_frozen(s, P, ps);
    if (!ps.miss) encode_pod(s, P, ps);
    miss = ps.miss;
  } catch (const EncodeError&) {
    miss = true;
  }
  e.prog.resize(prog0);
  e.pods.resize(pods0);
  s->req_cache.resize(caches0);
  s->pts_cache.resize(caches0);
  s->owned_templates.resize(caches0);
  s->pod_selectors.resize(caches0);
  s->tmpl_match.resize(caches0);
  e.prefilter_names.erase(P);
  e.prefilter_reject.erase(P);
  s->pods.pop_back();
  return miss;
}

// The hints announced since the last check: a full re-encode only when one of
// them extends the universe (a hint alone no longer forces one).
int check_hints(ksg_snapshot* s, int32_t* appended) {
  for (; s->hints_seen < s->hints.size(); s->hints_seen++)
    if (extends_universe(s, s->hints[s->hints_seen])) {
      if (appended) *appended = 0;
      return do_encode(s);
    }
  return KSG_OK;
}

int encode_incremental(ksg_snapshot* s, int32_t* appended) {
  if (appended) *appended = 0;
  if (!s->encoded) return do_encode(s);
  const int P = (int)s->pods.size();
  if (s->n_encoded == P) {
    if (appended) *appended = 1;
    return check_hints(s, appended);
  }
  Encoded& e = s->e;
  const size_t prog0 = e.prog.size(), pods0 = e.pods.size(), caches0 = s->req_cache.size();
  bool miss = false;
  try {
    for (int i = s->n_encoded; i < P && !miss; i++) {
      Pass ps{s, true};
      prepare_frozen(s, i, ps);
      if (!ps.miss) encode_pod(s, i, ps);
      miss = ps.miss;
    }
  } catch (const EncodeError& x) {
    miss = true;
  }
  if (miss) {
    e.prog.resize(prog0);
    e.pods.resize(pods0);
    for (auto* v : {&s->req_cache}) v->resize(caches0);
    s->pts_cache.resize(caches0);
    s->owned_templates.resize(caches0);
    s->pod_selectors.resize(caches0);
    s->tmpl_match.resize(caches0);
    return do_encode(s);
  }
  finish_arrays(s);
  s->n_encoded = P;
  if (appended) *appended = 1;
  return check_hints(s, appended);
}

// Upload the current encoding and replay the bindings.
int upload_all(ksg_snapshot* s, ksg_ctx* ctx) {
  int rc;
  ksg_nodes nd;
  ksg_topology tp;
  ksg_workload wl;
  ksg_profile pf;
  fill_views(s, &nd, &tp, &wl, &pf);
  auto dev = [&](int r, const char* what) {
    return fail(s, r, std::string(what) + ": " + ksg_last_error(ctx));
  };
  if ((rc = ksg_set_profile(ctx, &pf))) return dev(rc, "ksg_set_profile");
  if ((rc = ksg_load_nodes(ctx, &nd, &tp))) return dev(rc, "ksg_load_nodes");
  if ((rc = ksg_load_workload(ctx, &wl))) return dev(rc, "ksg_load_workload");
  if (!s->binds.empty()) {   // the bindings replayed in one launch
    std::vector<int32_t> bp, bn;
    for (auto& b : s->binds) {
      bp.push_back(b.first);
      bn.push_back(b.second);
    }
    if ((rc = ksg_commit_batch(ctx, bp.data(), bn.data(), (int32_t)bp.size())))
      return dev(rc, "ksg_commit_batch (replayed bindings)");
  }
  s->loaded_ctx = ctx;
  s->loaded_epoch = s->epoch;
  s->n_loaded = s->n_encoded;
  s->prog_loaded = s->e.prog.size();
  return KSG_OK;
}

int full_load(ksg_snapshot* s, ksg_ctx* ctx) {
  const int rc = do_encode(s);
  return rc ? rc : upload_all(s, ctx);
}

// Everything encode_pod would refuse for this pod alone, checked before the
// pod joins the snapshot: one unsupported pod must not make every later
// sync / encode of the snapshot fail.  Throws EncodeError.
void validate_pod(const ksg_snapshot* s, const Pod& p) {
  for (auto& c : p.spread) (void)canon_selector(c.sel);
  (void)canon_selector(p.default_sel);
  for (auto* v : {&p.aff_req, &p.aff_pref, &p.anti_req, &p.anti_pref})
    for (auto& t : *v) (void)term_scope(t, p);
  std::set<std::string> scal = s->scalars;
  for (auto& kv : pod_requests(p, false))
    if (is_scalar(kv.first)) scal.insert(kv.first);
  if (3 + scal.size() > (size_t)KSG_MAX_RES)
    throw EncodeError{KSG_E_UNSUPPORTED, "more than " + std::to_string(KSG_MAX_RES) + " resource columns"};
}

// ksg_snapshot_statuses' scan of one block of 64 nodes: stores the passed
// defaults (code Success, no message) and returns the rejected nodes as a
// bit mask (a word other than 0 / KSG_FS_NOT_EVALUATED).  (An AVX2 form was
// no faster: the pass is bound by its stores.)
uint64_t scan_block_sse2(const uint32_t* w, int32_t* code, int32_t* msg) {
  const __m128i v_pass = _mm_setzero_si128(), v_ne = _mm_set1_epi32((int)KSG_FS_NOT_EVALUATED);
  const __m128i v_ok = _mm_set1_epi32((int)KSG_CODE_SUCCESS), v_none = _mm_set1_epi32(-1);
  uint64_t mask = 0;
  for (int i = 0; i < 64; i += 4) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(w + i));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(code + i), v_ok);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(msg + i), v_none);
    const __m128i ok = _mm_or_si128(_mm_cmpeq_epi32(v, v_pass), _mm_cmpeq_epi32(v, v_ne));
    mask |= (uint64_t)(~_mm_movemask_ps(_mm_castsi128_ps(ok)) & 0xf) << i;
  }
  return mask;
}

// scan_block_sse2's mask without the stores (ksg_snapshot_statuses_kept's sparse form)
uint64_t mask_block_sse2(const uint32_t* w) {
  const __m128i v_pass = _mm_setzero_si128(), v_ne = _mm_set1_epi32((int)KSG_FS_NOT_EVALUATED);
  uint64_t mask = 0;
  for (int i = 0; i < 64; i += 4) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(w + i));
    const __m128i ok = _mm_or_si128(_mm_cmpeq_epi32(v, v_pass), _mm_cmpeq_epi32(v, v_ne));
    mask |= (uint64_t)(~_mm_movemask_ps(_mm_castsi128_ps(ok)) & 0xf) << i;
  }
  return mask;
}

// framework.Status (code, Message()) of a Filter status word at `node` for
// `pod`; msg may be null when only the code is wanted.
bool status_of(const Encoded& e, int32_t pod, uint32_t word, int32_t node, int* code, std::string* msg,
               std::string* err) {
  std::string m;
  int c = KSG_CODE_SUCCESS;
  const int pl = (int)(word & 0xffu) - 1;
  const uint32_t reason = word >> 8;
  if (word == KSG_FS_NOT_EVALUATED) {
    *err = "node not evaluated";
    return false;
  }
  switch (pl) {
    case -1:
      break;
    case KSG_PL_NODE_UNSCHEDULABLE:
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      if (msg) m = "node(s) were unschedulable";
      break;
    case KSG_PL_NODE_NAME:
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      if (msg) m = "node(s) didn't match the requested node name";
      break;
    case KSG_PL_TAINT_TOLERATION: {
      if ((int)reason >= e.max_taints) {
        *err = "taint slot";
        return false;
      }
      const uint32_t t = e.taints[(size_t)reason * e.N + node];
      if (t == 0) {
        *err = "empty taint slot";
        return false;
      }
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      if (msg) m = "node(s) had untolerated taint " + e.taint_strings[t - 1];
      break;
    }
    case KSG_PL_NODE_AFFINITY:
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      if (msg) m = "node(s) didn't match Pod's node affinity/selector";
      break;
    case KSG_PL_NODE_PORTS:
      c = KSG_CODE_UNSCHEDULABLE;
      if (msg) m = "node(s) didn't have free ports for the requested pod ports";
      break;
    case KSG_PL_NODE_RESOURCES_FIT: {
      // fitsRequest reason order: pods, cpu, memory, ephemeral, scalars;
      // Unresolvable when the request exceeds the allocatable outright.
      c = KSG_CODE_UNSCHEDULABLE;
      const ksg_pod& p = e.pods[pod];
      if (msg && (reason & 1u)) m = "Too many pods";
      for (size_t r = 0; r < e.res_names.size(); r++)
        if (reason & (1u << (r + 1))) {
          if (msg) m += (m.empty() ? "Insufficient " : ", Insufficient ") + e.res_names[r];
          if (p.req[r] > e.alloc[r * e.N + node]) c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
        }
      break;
    }
    case KSG_PL_POD_TOPOLOGY_SPREAD:
      c = reason == 1 ? KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE : KSG_CODE_UNSCHEDULABLE;
      if (msg)
        m = reason == 1 ? "node(s) didn't match pod topology spread constraints (missing required label)"
                        : "node(s) didn't match pod topology spread constraints";
      break;
    case KSG_PL_INTER_POD_AFFINITY:
      c = reason == 1 ? KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE : KSG_CODE_UNSCHEDULABLE;
      if (msg)
        m = reason == 1   ? "node(s) didn't match pod affinity rules"
            : reason == 2 ? "node(s) didn't match pod anti-affinity rules"
                          : "node(s) didn't satisfy existing pods anti-affinity rules";
      break;
    case KSG_PL_VOLUME_RESTRICTIONS:   // ErrReasonReadWriteOncePodConflict
      c = KSG_CODE_UNSCHEDULABLE;
      if (msg) m = "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode";
      break;
    case KSG_PL_VOLUME_BINDING: {   // FindPodVolumes' reasons, in order
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      static const char* const kVb[3] = {"node(s) had volume node affinity conflict",
                                         "node(s) didn't find available persistent volumes to bind",
                                         "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)"};
      for (int b = 0; msg && b < 3; b++)
        if (reason & (1u << b)) m += (m.empty() ? "" : ", ") + std::string(kVb[b]);
      break;
    }
    case KSG_PL_VOLUME_ZONE:
      c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
      if (msg) m = "node(s) had no available volume zone";
      break;
    default:
      *err = "unexpected word";
      return false;
  }
  *code = c;
  if (msg) *msg = std::move(m);
  return true;
}

}  // namespace

// ============================================================================
extern "C" {

int ksg_snapshot_new(const ksg_profile_view* pv, ksg_snapshot** out) {
  if (!pv || !out) return KSG_E_INVALID;
  *out = nullptr;
  ksg_snapshot* s = new ksg_snapshot();
  Profile& p = s->prof;
  for (int32_t i = 0; i < pv->n_plugins; i++) {
    std::string name = S(pv->plugins[i].name);
    p.plugins.emplace_back(name, pv->plugins[i].weight);
    const std::string key = plain_name(name);
    const int pid = plugin_id(key);
    if (pid >= 0) {
      p.enabled.push_back(pid);
    } else if (!non_eval(key)) {
      delete s;
      return KSG_E_UNSUPPORTED;   // not an in-tree Filter/Score plugin
    }
  }
  std::string perr;
  if (!derive_profile(p, pv, perr)) {
    delete s;
    return KSG_E_UNSUPPORTED;   // a per-point set the registry / framework refuses
  }
  p.fit_strategy = pv->fit_strategy ? S(pv->fit_strategy) : "LeastAllocated";
  if (p.fit_strategy != "LeastAllocated" && p.fit_strategy != "MostAllocated" &&
      p.fit_strategy != "RequestedToCapacityRatio") {
    delete s;
    return KSG_E_INVALID;   // not a scoring strategy
  }
  // the plugin-args validation of the scheduler (profile.py Profile.validate_args)
  if (p.fit_strategy == "RequestedToCapacityRatio") {
    if (pv->n_shape <= 0 || pv->n_shape > KSG_MAX_SHAPE || !pv->shape_utilization || !pv->shape_score) {
      delete s;
      return pv->n_shape > KSG_MAX_SHAPE ? KSG_E_UNSUPPORTED : KSG_E_INVALID;
    }
    for (int32_t i = 0; i < pv->n_shape; i++) {
      const int32_t u = pv->shape_utilization[i], sc = pv->shape_score[i];
      if (u < 0 || u > 100 || sc < 0 || sc > 10 || (i > 0 && u <= pv->shape_utilization[i - 1])) {
        delete s;
        return KSG_E_INVALID;
      }
      p.shape.emplace_back(u, sc);
    }
  }
  if (pv->n_default_constraints < 0 || (pv->n_default_constraints > 0 && !pv->default_constraints) ||
      (pv->n_default_constraints > 0 && pv->pts_system_defaulted)) {
    delete s;
    return KSG_E_INVALID;
  }
  std::set<std::pair<std::string, std::string>> seen;
  for (int32_t i = 0; i < pv->n_default_constraints; i++) {
    const ksg_spread_view& c = pv->default_constraints[i];
    Spread sp;
    sp.skew = c.max_skew;
    sp.key = S(c.topology_key);
    sp.when = S(c.when_unsatisfiable);
    sp.min_domains = c.min_domains;
    sp.nap = S(c.node_affinity_policy);
    sp.ntp = S(c.node_taints_policy);
    if (sp.skew <= 0 || sp.key.empty() || (sp.when != "DoNotSchedule" && sp.when != "ScheduleAnyway") ||
        c.selector.is_set || !seen.insert({sp.key, sp.when}).second) {
      delete s;
      return KSG_E_INVALID;
    }
    p.pts_defaults.push_back(std::move(sp));
  }
  for (int32_t i = 0; i < pv->n_fit_resources; i++)
    p.fit_res.emplace_back(S(pv->fit_resources[i].name), pv->fit_resources[i].value);
  for (int32_t i = 0; i < pv->n_ba_resources; i++)
    p.ba_res.emplace_back(S(pv->ba_resources[i].name), pv->ba_resources[i].value);
  for (int32_t i = 0; i < pv->n_fit_ignored_resources; i++) p.ignored.insert(S(pv->fit_ignored_resources[i]));
  for (int32_t i = 0; i < pv->n_fit_ignored_groups; i++) p.ignored_groups.insert(S(pv->fit_ignored_groups[i]));
  for (auto& r : p.fit_res)
    if (is_scalar(r.first)) s->scalars.insert(r.first);
  for (auto& r : p.ba_res)
    if (is_scalar(r.first)) s->scalars.insert(r.first);
  p.hard_weight = pv->hard_pod_affinity_weight;
  p.ignore_pref = pv->ignore_preferred_terms_of_existing_pods != 0;
  p.pts_system = pv->pts_system_defaulted != 0;
  p.ba_skip_be = pv->ba_skip_best_effort != 0;
  *out = s;
  return KSG_OK;
}

int ksg_snapshot_profile_info(ksg_snapshot* s, ksg_profile_info* out) {
  if (!s || !out) return KSG_E_INVALID;
  std::memset(out, 0, sizeof(*out));
  const Profile& p = s->prof;
  for (int pt = 0; pt < KSG_NPOINTS; pt++) {
    out->n_order[pt] = (int32_t)p.order[pt].size();
    for (size_t k = 0; k < p.order[pt].size(); k++) out->order[pt][k] = p.order[pt][k];
  }
  for (int pid = 0; pid < KSG_NPLUGINS; pid++) {
    out->store_weight[pid] = p.store_w[pid];
    out->selection_weight[pid] = p.sel_w[pid];
    if (kExt[pid][4]) out->normalize_mask |= 1u << pid;
  }
  return KSG_OK;
}

int ksg_snapshot_free(ksg_snapshot* s) {
  delete s;
  return KSG_OK;
}

const char* ksg_snapshot_error(ksg_snapshot* s) { return s ? s->err.c_str() : "null snapshot"; }

int ksg_snapshot_add_node(ksg_snapshot* s, const ksg_node_view* v, int32_t* index) {
  if (!s || !v || !v->name) return KSG_E_INVALID;
  Node n;
  n.name = v->name;
  if (s->node_index.count(n.name)) return fail(s, KSG_E_INVALID, "duplicate node name " + n.name);
  n.labels = copy_pairs(v->n_labels, v->labels);
  for (int32_t i = 0; i < v->n_taints; i++)
    n.taints.push_back(Taint{S(v->taints[i].key), S(v->taints[i].value), S(v->taints[i].effect)});
  n.alloc = copy_res(v->n_alloc, v->allocatable);
  n.unsched = v->unschedulable != 0;
  std::set<std::string> scal = s->scalars;
  for (auto& kv : n.alloc)
    if (is_scalar(kv.first)) scal.insert(kv.first);
  if (3 + scal.size() > (size_t)KSG_MAX_RES)
    return fail(s, KSG_E_UNSUPPORTED, "node " + n.name + ": more than " + std::to_string(KSG_MAX_RES) +
                                          " resource columns");
  s->scalars = std::move(scal);
  for (int32_t i = 0; i < v->n_images; i++) {
    Image im;
    for (int32_t k = 0; k < v->images[i].n_names; k++) im.names.push_back(S(v->images[i].names[k]));
    im.size = v->images[i].size_bytes;
    n.images.push_back(std::move(im));
  }
  const int32_t idx = (int32_t)s->nodes.size();
  s->node_index[n.name] = idx;
  s->nodes.push_back(std::move(n));
  s->encoded = false;
  s->loaded_ctx = nullptr;   // the node set changed: the next sync reloads
  if (index) *index = idx;
  return KSG_OK;
}

namespace {
// framework.AffinityTerm matches Namespaces ∪ {ns : namespaceSelector matches
// its labels} [upstream interpodaffinity mergeAffinityTermNamespacesIfNotEmpty,
// v1.32]: the selector becomes the list of the snapshot's namespaces it
// matches (ingest.py _affinity_term).  Returns whether `t.ns` changed.
bool resolve_term(const ksg_snapshot* s, AffTerm& t) {
  if (!t.resolved) {
    if (!t.ns_sel.set || t.ns_sel.empty()) return false;
    t.resolved = true;
    t.ns_given = t.ns;
    t.ns_req = t.ns_sel;
    t.ns_sel = Sel{};
  }
  const Canon c = canon_selector(t.ns_req);
  std::set<std::string> ns(t.ns_given.begin(), t.ns_given.end());
  for (auto& kv : s->namespaces)
    if (selector_matches(c, kv.second)) ns.insert(kv.first);
  std::vector<std::string> out(ns.begin(), ns.end());
  if (out.empty()) out = {kNoNamespace};
  if (out == t.ns) return false;
  t.ns = std::move(out);
  return true;
}

bool resolve_namespaces(const ksg_snapshot* s, Pod& p) {
  bool changed = false;
  for (auto* v : {&p.aff_req, &p.aff_pref, &p.anti_req, &p.anti_pref})
    for (auto& t : *v)
      if (t.resolved || (t.ns_sel.set && !t.ns_sel.empty())) {
        if (!s->have_namespaces)
          throw EncodeError{KSG_E_UNSUPPORTED,
                            "namespaceSelector with requirements needs the snapshot's namespaces "
                            "(ksg_snapshot_add_namespace)"};
        changed = resolve_term(s, t) || changed;
      }
  return changed;
}
}  // namespace

int ksg_snapshot_add_pv(ksg_snapshot* s, const ksg_pv_view* v) {
  if (!s || !v || !v->name || v->n_labels < 0 || v->n_terms < 0) return KSG_E_INVALID;
  PV pv;
  pv.name = v->name;
  pv.labels = copy_pairs(v->n_labels, v->labels);
  pv.storage_class = S(v->storage_class);
  pv.has_claim_ref = v->claim_name != nullptr;
  pv.claim_ns = S(v->claim_namespace);
  pv.claim_name = S(v->claim_name);
  pv.source = S(v->source);
  pv.has_na = v->has_node_affinity != 0;
  for (int32_t i = 0; i < v->n_terms; i++) pv.na.push_back(copy_term(v->terms[i]));
  s->pvs[pv.name] = std::move(pv);
  s->encoded = false;        // every pod's claims resolve again at the next (full) encode
  s->loaded_ctx = nullptr;
  return KSG_OK;
}

int ksg_snapshot_add_pvc(ksg_snapshot* s, const ksg_pvc_view* v) {
  if (!s || !v || !v->name || v->n_access_modes < 0 || v->n_annotations < 0) return KSG_E_INVALID;
  PVC c;
  c.ns = v->namespace_ ? S(v->namespace_) : "default";
  c.name = v->name;
  c.volume_name = S(v->volume_name);
  c.storage_class = S(v->storage_class);
  for (int32_t i = 0; i < v->n_access_modes; i++) c.modes.push_back(S(v->access_modes[i]));
  c.ann = copy_pairs(v->n_annotations, v->annotations);
  c.deleting = v->deleting != 0;
  s->pvcs[{c.ns, c.name}] = std::move(c);
  s->encoded = false;
  s->loaded_ctx = nullptr;
  return KSG_OK;
}

int ksg_snapshot_add_storage_class(ksg_snapshot* s, const ksg_storage_class_view* v) {
  if (!s || !v || !v->name || v->n_allowed_topologies < 0) return KSG_E_INVALID;
  SClass c;
  c.name = v->name;
  c.provisioner = S(v->provisioner);
  c.mode = (v->binding_mode && *v->binding_mode) ? S(v->binding_mode) : std::string("Immediate");
  for (int32_t i = 0; i < v->n_allowed_topologies; i++) {
    const ksg_topology_term_view& t = v->allowed_topologies[i];
    std::vector<std::pair<std::string, std::vector<std::string>>> term;
    for (int32_t k = 0; k < t.n_requirements; k++) {
      std::vector<std::string> vals;
      for (int32_t j = 0; j < t.requirements[k].n_values; j++) vals.push_back(S(t.requirements[k].values[j]));
      term.emplace_back(S(t.requirements[k].key), std::move(vals));
    }
    c.topo.push_back(std::move(term));
  }
  s->classes[c.name] = std::move(c);
  s->encoded = false;
  s->loaded_ctx = nullptr;
  return KSG_OK;
}

int ksg_snapshot_clear_storage(ksg_snapshot* s) {
  if (!s) return KSG_E_INVALID;
  if (s->pvs.empty() && s->pvcs.empty() && s->classes.empty()) return KSG_OK;
  s->pvs.clear();
  s->pvcs.clear();
  s->classes.clear();
  s->encoded = false;   // claims resolve again (a deleted object's claims now fail) at the next encode
  s->loaded_ctx = nullptr;
  return KSG_OK;
}

int ksg_snapshot_add_namespace(ksg_snapshot* s, const char* name, int32_t n_labels, const ksg_str_pair* labels) {
  if (!s || !name || n_labels < 0 || (n_labels > 0 && !labels)) return KSG_E_INVALID;
  s->namespaces[S(name)] = copy_pairs(n_labels, labels);
  s->have_namespaces = true;
  // re-resolve the selectors already taken in; a change invalidates the
  // encoding (next sync re-encodes in full)
  bool changed = false;
  try {
    for (auto& p : s->pods) changed = resolve_namespaces(s, p) || changed;
    for (auto& h : s->hints) changed = resolve_namespaces(s, h) || changed;
  } catch (const EncodeError& x) {
    return fail(s, x.code, x.msg);
  }
  if (changed) s->encoded = false;
  return KSG_OK;
}

namespace {
// A pod view into the snapshot's Pod, validated (ksg_snapshot_add_pod /
// ksg_snapshot_hint_pod).  Returns 0 or the failing code (message set).
int pod_from_view(ksg_snapshot* s, const ksg_pod_view* v, Pod& p) {
  p.ns = v->namespace_ ? S(v->namespace_) : "default";
  p.name = S(v->name);
  p.labels = copy_pairs(v->n_labels, v->labels);
  p.containers = copy_containers(v->n_containers, v->containers);
  p.init = copy_containers(v->n_init_containers, v->init_containers);
  p.has_overhead = v->has_overhead != 0;
  p.overhead = copy_res(v->n_overhead, v->overhead);
  p.node_name = S(v->node_name);
  p.has_node_selector = v->has_node_selector != 0;
  p.node_selector = copy_pairs(v->n_node_selector, v->node_selector);
  p.has_na_req = v->has_na_required != 0;
  for (int32_t i = 0; i < v->n_na_required; i++) p.na_req.push_back(copy_term(v->na_required[i]));
  p.has_na_pref = v->has_na_preferred != 0;
  for (int32_t i = 0; i < v->n_na_preferred; i++)
    p.na_pref.push_back(PrefTerm{v->na_preferred[i].weight, copy_term(v->na_preferred[i].preference)});
  p.aff_req = copy_aff(v->n_pod_affinity_required, v->pod_affinity_required);
  p.aff_pref = copy_aff(v->n_pod_affinity_preferred, v->pod_affinity_preferred);
  p.anti_req = copy_aff(v->n_pod_anti_affinity_required, v->pod_anti_affinity_required);
  p.anti_pref = copy_aff(v->n_pod_anti_affinity_preferred, v->pod_anti_affinity_preferred);
  for (int32_t i = 0; i < v->n_tolerations; i++)
    p.tols.push_back(Tol{S(v->tolerations[i].key), S(v->tolerations[i].op), S(v->tolerations[i].value),
                         S(v->tolerations[i].effect)});
  for (int32_t i = 0; i < v->n_spread; i++) {
    const ksg_spread_view& c = v->spread[i];
    Spread sp;
    sp.skew = c.max_skew;
    sp.key = S(c.topology_key);
    sp.when = S(c.when_unsatisfiable);
    sp.sel = copy_sel(c.selector);
    sp.min_domains = c.min_domains;
    sp.nap = S(c.node_affinity_policy);
    sp.ntp = S(c.node_taints_policy);
    for (int32_t k = 0; k < c.n_match_label_keys; k++) sp.mlk.push_back(S(c.match_label_keys[k]));
    p.spread.push_back(std::move(sp));
  }
  p.default_sel = copy_sel(v->default_spread_selector);
  p.terminating = v->terminating != 0;
  p.priority = v->priority;
  // volumes whose source makes a volume plugin's PreFilter run (include/
  // ksched_snapshot.h ksg_volume_view; model.Pod.volumes_needing_plugins):
  // refused while any volume plugin runs at PreFilter or Filter
  if (v->n_volumes < 0 || (v->n_volumes > 0 && !v->volumes)) return KSG_E_INVALID;
  bool vol_run = false;
  for (int pt : {KSG_POINT_PREFILTER, KSG_POINT_FILTER})
    for (int pid : s->prof.order[pt])
      vol_run = vol_run || pid == KSG_PL_VOLUME_RESTRICTIONS || pid == KSG_PL_NODE_VOLUME_LIMITS ||
                pid == KSG_PL_VOLUME_BINDING || pid == KSG_PL_VOLUME_ZONE;
  for (int32_t i = 0; i < v->n_volumes; i++) {
    static const char* const kRefused[] = {"ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "azureDisk",
                                           "azureFile", "cinder", "vsphereVolume", "portworxVolume", "rbd", "iscsi"};
    const std::string kind = S(v->volumes[i].kind);
    if (kind == "persistentVolumeClaim") p.claims.push_back(S(v->volumes[i].claim_name));
    for (const char* k : kRefused)
      if (vol_run && kind == k)
        return fail(s, KSG_E_UNSUPPORTED,
                    "pod " + p.ns + "/" + p.name + ": volume '" + S(v->volumes[i].name) + "' (" + kind +
                        ") makes the volume plugins' PreFilter run; of the volume sources only "
                        "persistentVolumeClaim is modelled");
  }
  try {
    resolve_namespaces(s, p);
    validate_pod(s, p);
  } catch (const EncodeError& x) {
    return fail(s, x.code, "pod " + p.ns + "/" + p.name + ": " + x.msg);
  }
  return KSG_OK;
}
}  // namespace

std::string hint_key(const std::string& ns, const std::string& name) { return ns + '/' + name; }

void hint_swap(ksg_snapshot* s, size_t i, size_t j) {
  if (i == j) return;
  std::swap(s->hints[i], s->hints[j]);
  s->hint_index[hint_key(s->hints[i].ns, s->hints[i].name)] = i;
  s->hint_index[hint_key(s->hints[j].ns, s->hints[j].name)] = j;
}

// Forget the hint of pod ns/name, if any (the pod was added or deleted), in
// O(1): swapped to the end and popped.  A hint inside the probed prefix
// [0, hints_seen) first trades places with the prefix's last entry, so the
// entry that lands at the prefix boundary is re-probed (a seen hint probes
// clean, so that costs one probe, never a result).  The current encoding
// keeps what the hint brought in until the next full encode.
void drop_hint(ksg_snapshot* s, const std::string& ns, const std::string& name) {
  auto it = s->hint_index.find(hint_key(ns, name));
  if (it == s->hint_index.end()) return;
  size_t k = it->second;
  if (k < s->hints_seen) {
    hint_swap(s, k, s->hints_seen - 1);
    k = --s->hints_seen;
  }
  hint_swap(s, k, s->hints.size() - 1);
  s->hint_index.erase(hint_key(ns, name));
  s->hints.pop_back();
}

int ksg_snapshot_add_pod(ksg_snapshot* s, const ksg_pod_view* v, int32_t* index) {
  if (!s || !v || !v->name) return KSG_E_INVALID;
  Pod p;
  const int rc = pod_from_view(s, v, p);
  if (rc) return rc;
  for (auto& kv : pod_requests(p, false))
    if (is_scalar(kv.first)) s->scalars.insert(kv.first);
  drop_hint(s, p.ns, p.name);   // the pod itself now keeps its terms in the universe
  const int32_t idx = (int32_t)s->pods.size();
  s->pods.push_back(std::move(p));
  if (index) *index = idx;
  return KSG_OK;
}

int ksg_snapshot_hint_pod(ksg_snapshot* s, const ksg_pod_view* v) {
  if (!s || !v || !v->name) return KSG_E_INVALID;
  Pod p;
  const int rc = pod_from_view(s, v, p);
  if (rc) return rc;
  for (auto& kv : pod_requests(p, false))
    if (is_scalar(kv.first)) s->scalars.insert(kv.first);
  drop_hint(s, p.ns, p.name);   // announced again: the newer spec replaces the older
  s->hint_index[hint_key(p.ns, p.name)] = s->hints.size();
  s->hints.push_back(std::move(p));
  return KSG_OK;
}

int ksg_snapshot_unhint_pod(ksg_snapshot* s, const char* ns, const char* name) {
  if (!s || !name) return KSG_E_INVALID;
  drop_hint(s, ns ? ns : "default", name);   // pod_from_view's defaulting
  return KSG_OK;
}

int ksg_snapshot_bind(ksg_snapshot* s, int32_t pod, int32_t node) {
  if (!s) return KSG_E_INVALID;
  if (pod < 0 || pod >= (int32_t)s->pods.size() || node < 0 || node >= (int32_t)s->nodes.size())
    return fail(s, KSG_E_INVALID, "bind: index out of range");
  s->binds.emplace_back(pod, node);
  s->loaded_ctx = nullptr;   // bindings are replayed by the next load
  return KSG_OK;
}

int ksg_snapshot_node_index(ksg_snapshot* s, const char* name, int32_t* index) {
  if (!s || !name || !index) return KSG_E_INVALID;
  auto it = s->node_index.find(name);
  *index = it == s->node_index.end() ? -1 : it->second;
  return KSG_OK;
}

int ksg_snapshot_encode(ksg_snapshot* s) {
  if (!s) return KSG_E_INVALID;
  if (s->nodes.empty()) return fail(s, KSG_E_STATE, "no nodes");
  return do_encode(s);
}

int ksg_snapshot_view(ksg_snapshot* s, ksg_nodes* nd, ksg_topology* tp, ksg_workload* wl, ksg_profile* pf) {
  if (!s) return KSG_E_INVALID;
  if (!s->encoded || s->n_encoded != (int)s->pods.size())
    return fail(s, KSG_E_STATE, "snapshot not encoded (pods added since the last encode)");
  fill_views(s, nd, tp, wl, pf);
  return KSG_OK;
}

int ksg_snapshot_load(ksg_snapshot* s, ksg_ctx* ctx) {
  if (!s || !ctx) return KSG_E_INVALID;
  if (s->nodes.empty()) return fail(s, KSG_E_STATE, "no nodes");
  return full_load(s, ctx);
}

int ksg_snapshot_encode_incremental(ksg_snapshot* s, int32_t* appended) {
  if (!s) return KSG_E_INVALID;
  if (s->nodes.empty()) return fail(s, KSG_E_STATE, "no nodes");
  return encode_incremental(s, appended);
}

int ksg_snapshot_sync(ksg_snapshot* s, ksg_ctx* ctx, int32_t* appended) {
  if (!s || !ctx) return KSG_E_INVALID;
  if (appended) *appended = 0;
  if (s->nodes.empty()) return fail(s, KSG_E_STATE, "no nodes");
  if (s->loaded_ctx != ctx) return full_load(s, ctx);
  int rc = encode_incremental(s, nullptr);
  if (rc) return rc;
  if (s->loaded_epoch != s->epoch) return upload_all(s, ctx);   // the universe changed
  const int P = s->n_encoded;
  Encoded& e = s->e;
  if (s->n_loaded < P) {
    ksg_workload tail{};
    tail.pods = e.pods.data() + s->n_loaded;
    tail.n_pods = P - s->n_loaded;
    tail.prog = e.prog.data() + s->prog_loaded;
    tail.prog_len = (int64_t)(e.prog.size() - s->prog_loaded);
    rc = ksg_append_pods(ctx, &tail, (int64_t)s->prog_loaded);
    if (rc) return fail(s, rc, std::string("ksg_append_pods: ") + ksg_last_error(ctx));
    s->n_loaded = P;
    s->prog_loaded = e.prog.size();
  }
  if (appended) *appended = 1;
  return KSG_OK;
}

int ksg_snapshot_assume(ksg_snapshot* s, ksg_ctx* ctx, int32_t pod, int32_t node) {
  if (!s || !ctx) return KSG_E_INVALID;
  if (s->loaded_ctx != ctx || pod >= s->n_loaded) return fail(s, KSG_E_STATE, "assume: sync the context first");
  const int rc = ksg_commit(ctx, pod, node);
  if (rc) return fail(s, rc, std::string("ksg_commit: ") + ksg_last_error(ctx));
  s->binds.emplace_back(pod, node);
  return KSG_OK;
}

int ksg_snapshot_forget(ksg_snapshot* s, ksg_ctx* ctx, int32_t pod, int32_t node) {
  if (!s || !ctx) return KSG_E_INVALID;
  auto it = std::find(s->binds.begin(), s->binds.end(), std::make_pair(pod, node));
  if (it == s->binds.end()) return fail(s, KSG_E_INVALID, "forget: no such binding");
  if (s->loaded_ctx == ctx) {
    const int rc = ksg_uncommit(ctx, pod, node);
    if (rc) return fail(s, rc, std::string("ksg_uncommit: ") + ksg_last_error(ctx));
  }
  s->binds.erase(it);
  return KSG_OK;
}

int ksg_snapshot_status(ksg_snapshot* s, int32_t pod, uint32_t word, int32_t node, int32_t* code, char* msg,
                        int32_t cap, int32_t* len) {
  if (!s || !code) return KSG_E_INVALID;
  if (!s->encoded || pod < 0 || pod >= (int32_t)s->e.pods.size() || node < 0 || node >= s->e.N)
    return fail(s, KSG_E_INVALID, "status: index out of range");
  std::string m, err;
  int c;
  if (!status_of(s->e, pod, word, node, &c, &m, &err)) return fail(s, KSG_E_INVALID, "status: " + err);
  *code = c;
  if (len) *len = (int32_t)m.size();
  if (msg && cap > 0) {
    const size_t n = std::min<size_t>(m.size(), (size_t)cap - 1);
    std::memcpy(msg, m.data(), n);
    msg[n] = 0;
  }
  return KSG_OK;
}

// ksg_snapshot_statuses and its delta form: dense stores the passed defaults
// of every node; otherwise only the rejected nodes are written.  rej (or
// null) collects the rejected nodes.
static int statuses_impl(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes, int32_t* code,
                         int32_t* msg, char* buf, int64_t cap, int32_t* n_msgs, int64_t* len, bool dense,
                         std::vector<int32_t>* rej);

int ksg_snapshot_statuses(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes, int32_t* code,
                          int32_t* msg, char* buf, int64_t cap, int32_t* n_msgs, int64_t* len) {
  return statuses_impl(s, pod, words, n_nodes, code, msg, buf, cap, n_msgs, len, true, nullptr);
}

int ksg_snapshot_statuses_kept(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes,
                               const int32_t** code, const int32_t** msg, char* buf, int64_t cap, int32_t* n_msgs,
                               int64_t* len) {
  if (!s || !code || !msg) return KSG_E_INVALID;
  *code = *msg = nullptr;
  if (n_nodes < 0) return fail(s, KSG_E_INVALID, "statuses: index out of range");
  auto& d = s->skept;
  // The arrays are the snapshot's own and read-only to the caller, so after a
  // complete call they hold exactly its output: the next call resets the
  // nodes that call rejected and writes only its own rejected nodes.  (The
  // sparse form pays per rejected node: past an eighth of the nodes rejected
  // by the last call, the dense pass is the cheaper one; measured on
  // configs[1] ~30 % rejected, configs[2] ~15 %.)
  const bool sparse = d.valid && d.code.size() == (size_t)n_nodes && d.rej.size() * 8 <= (size_t)n_nodes;
  if (d.code.size() != (size_t)n_nodes) {
    d.code.assign((size_t)n_nodes, KSG_CODE_SUCCESS);
    d.msg.assign((size_t)n_nodes, -1);
  }
  if (sparse)
    for (int32_t n : d.rej) {
      d.code[n] = KSG_CODE_SUCCESS;
      d.msg[n] = -1;
    }
  d.valid = false;   // (set again only when this call completes)
  d.rej.clear();
  (sparse ? d.sparse_calls : d.dense_calls)++;
  const int rc = statuses_impl(s, pod, words, n_nodes, d.code.data(), d.msg.data(), buf, cap, n_msgs, len, !sparse,
                               &d.rej);
  if (rc != KSG_OK) return rc;
  d.valid = true;
  *code = d.code.data();
  *msg = d.msg.data();
  return KSG_OK;
}

int ksg_snapshot_statuses_kept_stats(ksg_snapshot* s, int64_t* sparse_calls, int64_t* dense_calls) {
  if (!s) return KSG_E_INVALID;
  if (sparse_calls) *sparse_calls = s->skept.sparse_calls;
  if (dense_calls) *dense_calls = s->skept.dense_calls;
  return KSG_OK;
}

static int statuses_impl(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes, int32_t* code,
                         int32_t* msg, char* buf, int64_t cap, int32_t* n_msgs, int64_t* len, bool dense,
                         std::vector<int32_t>* rej) {
  if (!s || !words || !code || !msg) return KSG_E_INVALID;
  if (!s->encoded || pod < 0 || pod >= (int32_t)s->e.pods.size() || n_nodes != s->e.N)
    return fail(s, KSG_E_INVALID, "statuses: index out of range");
  const Encoded& e = s->e;
  // distinct messages: keyed by the word, plus the taint id for TaintToleration.
  // A key's message and code depend on nothing else (the taint strings and
  // resource names change only with a full encode), except NodeResourcesFit's
  // code, recomputed per node below (a request above the node's allocatable
  // is unresolvable).  So keys are formatted once per encoding, not per pod;
  // a call numbers the keys it meets in first-seen order.  Neighbouring nodes
  // mostly repeat a word: last-key shortcut, then a direct-mapped cache.
  auto& sc = s->status;
  if (sc.epoch != s->epoch) {
    sc.ids.clear();
    sc.msgs.clear();
    sc.codes.clear();
    sc.stamp.clear();
    sc.local.clear();
    for (int i = 0; i < sc.kDm; i++) sc.dm_key[i] = ~0ull;
    sc.epoch = s->epoch;
  }
  if (++sc.gen == 0) {   // stamp wrap: forget every call's stamp
    std::fill(sc.stamp.begin(), sc.stamp.end(), 0u);
    sc.gen = 1;
  }
  const uint32_t gen = sc.gen;
  sc.order.clear();
  const ksg_pod& p = e.pods[pod];
  uint64_t last_key = ~0ull;
  int32_t last_idx = -1;
  std::string err;
  // Most nodes pass: each block of 64 nodes stores the passed defaults and
  // yields its rejected nodes as a 64-bit mask in the same pass; the rejected
  // nodes are then decoded one by one.
  constexpr int32_t kB = 64;
  const uint32_t* taints = e.taints.data();
  const size_t N = (size_t)e.N;
  const uint32_t max_taints = (uint32_t)std::max(e.max_taints, 0);
  int32_t last_code = 0;
  for (int32_t b = 0; b < n_nodes; b += kB) {
    const int32_t m = std::min(kB, n_nodes - b);
    uint64_t mask = 0;   // the block's rejected nodes: four words per compare
    if (m == kB) {
      mask = dense ? scan_block_sse2(words + b, code + b, msg + b) : mask_block_sse2(words + b);
    } else {
      for (int32_t i = 0; i < m; i++) {
        const uint32_t w = words[b + i];
        if (dense) {
          code[b + i] = KSG_CODE_SUCCESS;
          msg[b + i] = -1;
        }
        mask |= (uint64_t)(w != 0 && w != KSG_FS_NOT_EVALUATED) << i;
      }
    }
    for (; mask; mask &= mask - 1) {
    const int32_t n = b + __builtin_ctzll(mask);
    const uint32_t w = words[n];
    const int pl = (int)(w & 0xffu) - 1;
    uint64_t key = w;
    if (pl == KSG_PL_TAINT_TOLERATION && (w >> 8) < max_taints) key |= (uint64_t)taints[(w >> 8) * N + n] << 32;
    if (key != last_key) {
      int32_t id;
      const int slot = (int)((key * 0x9E3779B97F4A7C15ull) >> 56);
      if (sc.dm_key[slot] == key) {
        id = sc.dm_id[slot];
      } else {
        auto it = sc.ids.find(key);
        if (it == sc.ids.end()) {
          std::string m;
          int c;
          if (!status_of(e, pod, w, n, &c, &m, &err)) return fail(s, KSG_E_INVALID, "statuses: " + err);
          it = sc.ids.emplace(key, (int32_t)sc.msgs.size()).first;
          sc.msgs.push_back(std::move(m));
          sc.codes.push_back(c);
          sc.stamp.push_back(0u);
          sc.local.push_back(-1);
        }
        id = it->second;
        sc.dm_key[slot] = key;
        sc.dm_id[slot] = id;
      }
      if (sc.stamp[id] != gen) {
        sc.stamp[id] = gen;
        sc.local[id] = (int32_t)sc.order.size();
        sc.order.push_back(id);
      }
      last_key = key;
      last_idx = sc.local[id];
      last_code = sc.codes[id];
    }
    int c = last_code;
    if (pl == KSG_PL_NODE_RESOURCES_FIT) {   // status_of's Fit code, per node
      const uint32_t reason = w >> 8;
      c = KSG_CODE_UNSCHEDULABLE;
      for (size_t r = 0; r < e.res_names.size(); r++)
        if ((reason & (1u << (r + 1))) && p.req[r] > e.alloc[r * N + n]) c = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;
    }
    code[n] = c;
    msg[n] = last_idx;
    if (rej) rej->push_back(n);
    }
  }
  int64_t total = 0;
  for (int32_t id : sc.order) total += (int64_t)sc.msgs[id].size() + 1;
  if (n_msgs) *n_msgs = (int32_t)sc.order.size();
  if (len) *len = total;
  if (buf && cap >= total) {
    char* o = buf;
    for (int32_t id : sc.order) {
      const std::string& m = sc.msgs[id];
      std::memcpy(o, m.data(), m.size());
      o += m.size();
      *o++ = 0;
    }
  }
  return KSG_OK;
}

int ksg_snapshot_prefilter(ksg_snapshot* s, int32_t pod, int32_t plugin, uint32_t result_status, int32_t* code,
                           int32_t* has_result, const char** names, int32_t cap, int32_t* n_names) {
  if (!s || !code) return KSG_E_INVALID;
  if (!s->encoded || pod < 0 || pod >= (int32_t)s->e.pods.size() || plugin < 0 || plugin >= KSG_NPLUGINS)
    return fail(s, KSG_E_INVALID, "prefilter: index out of range");
  const ksg_pod& p = s->e.pods[pod];
  if (has_result) *has_result = 0;
  if (n_names) *n_names = 0;
  uint32_t fskip = p.filter_skip;
  if (result_status & KSG_ST_IPA_PREFILTER_SKIP) fskip |= 1u << KSG_PL_INTER_POD_AFFINITY;
  auto rj = s->e.prefilter_reject.find(pod);
  if ((p.flags & KSG_POD_PREFILTER_REJECT) && rj != s->e.prefilter_reject.end() && rj->second.first == plugin &&
      !rj->second.second.empty()) {
    *code = KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE;   // its message: ksg_snapshot_prefilter_message
    return KSG_OK;
  }
  if ((fskip >> plugin) & 1u) {
    *code = KSG_CODE_SKIP;
    return KSG_OK;
  }
  *code = KSG_CODE_SUCCESS;
  auto pn = s->e.prefilter_names.find(pod);
  if (pn != s->e.prefilter_names.end()) {
    auto it = pn->second.find(plugin);
    if (it != pn->second.end()) {
      const auto& nm = it->second;
      if (has_result) *has_result = 1;
      if (n_names) *n_names = (int32_t)nm.size();
      if (names)
        for (int32_t k = 0; k < cap && k < (int32_t)nm.size(); k++) names[k] = nm[k].c_str();
    }
  }
  return KSG_OK;
}

int ksg_snapshot_prefilter_message(ksg_snapshot* s, int32_t pod, int32_t plugin, char* msg, int32_t cap,
                                   int32_t* len) {
  if (!s || !len) return KSG_E_INVALID;
  if (!s->encoded || pod < 0 || pod >= (int32_t)s->e.pods.size() || plugin < 0 || plugin >= KSG_NPLUGINS)
    return fail(s, KSG_E_INVALID, "prefilter_message: index out of range");
  std::string m;
  auto rj = s->e.prefilter_reject.find(pod);
  if ((s->e.pods[pod].flags & KSG_POD_PREFILTER_REJECT) && rj != s->e.prefilter_reject.end() &&
      rj->second.first == plugin)
    m = rj->second.second;
  *len = (int32_t)m.size();
  if (msg && cap > 0) {
    const size_t n = std::min<size_t>(m.size(), (size_t)cap - 1);
    std::memcpy(msg, m.data(), n);
    msg[n] = 0;
  }
  return KSG_OK;
}

int ksg_snapshot_counts(ksg_snapshot* s, int32_t* n_nodes, int32_t* n_pods, int32_t* n_res, int32_t* n_taint_vocab) {
  if (!s) return KSG_E_INVALID;
  if (n_nodes) *n_nodes = (int32_t)s->nodes.size();
  if (n_pods) *n_pods = (int32_t)s->pods.size();
  if (n_res) *n_res = s->encoded ? (int32_t)s->e.res_names.size() : 0;
  if (n_taint_vocab) *n_taint_vocab = s->encoded ? (int32_t)s->e.taint_vocab.size() : 0;
  return KSG_OK;
}

int ksg_snapshot_names(ksg_snapshot* s, const char** node, const char** res, const char** taint) {
  if (!s) return KSG_E_INVALID;
  if (!s->encoded) return fail(s, KSG_E_STATE, "snapshot not encoded");
  if (node)
    for (size_t i = 0; i < s->nodes.size(); i++) node[i] = s->nodes[i].name.c_str();
  if (res)
    for (size_t i = 0; i < s->e.res_names.size(); i++) res[i] = s->e.res_names[i].c_str();
  if (taint)
    for (size_t i = 0; i < s->e.taint_strings.size(); i++) taint[i] = s->e.taint_strings[i].c_str();
  return KSG_OK;
}

}  // extern "C"
