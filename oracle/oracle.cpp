// ORACLE — test infrastructure and CPU baseline only.  Never linked into the
// product library (libksched.so); only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg load liboracle.so.
//
// C++ restatement of the kube-scheduler v1.32 Filter/Score cycle, run over the
// same encoded snapshot the HIP kernels read (include/ksched.h), but with the
// reference's algorithm: every PodTopologySpread / InterPodAffinity PreFilter
// and PreScore rescans the pods on every node, exactly as the upstream
// plugins do per scheduling cycle;
// the device instead keeps incremental count tables.  Node loops run on
// OpenMP threads the way the upstream Parallelizer runs 16 goroutines.
//
// Parity: restated from the upstream design — the
// upstream source (k8s.io/kubernetes v1.32.5) is not in this container and
// cannot be built (no Go toolchain).  This restatement is
// pinned by (1) the independent pure-Python restatement oracle/pyoracle.py,
// which works on the unencoded object model, (2) the README known-answer test
// (README.md:56-81), and (3) the wrapper/store contract of the reference tests.
// Against the Go binary itself: parity unpinned.
//
// Upstream functions restated (all [upstream] pkg/scheduler/...):
//   framework/plugins/noderesources/fit.go            fitsRequest, Fit.Score
//   framework/plugins/noderesources/resource_allocation.go  calculateResourceAllocatableRequest
//   framework/plugins/noderesources/least_allocated.go / most_allocated.go
//   framework/plugins/noderesources/balanced_allocation.go  balancedResourceScorer
//   framework/plugins/tainttoleration/taint_toleration.go   Filter, Score, NormalizeScore
//   framework/plugins/nodeaffinity/node_affinity.go         PreFilter, Filter, Score
//   framework/plugins/nodeunschedulable, nodename            Filter
//   framework/plugins/imagelocality/image_locality.go       Score
//   framework/plugins/podtopologyspread/{filtering,scoring,common}.go
//   framework/plugins/interpodaffinity/{filtering,scoring}.go
//   framework/plugins/helper/normalize_score.go              DefaultNormalizeScore
//   framework/runtime/framework.go   RunFilterPlugins (first rejection ends a node),
//                                    RunScorePlugins (normalise, range check, weights)
//   schedule_one.go                  1 feasible node -> no scoring; selectHost
//                                    (tie-break made deterministic: lowest node index)

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <set>
#include <vector>

#include <omp.h>

#include "../include/ksched.h"

namespace {

constexpr int64_t kMaxNodeScore = 100;
constexpr int64_t kMB = 1024 * 1024;
constexpr int64_t kMinThreshold = 23 * kMB;
constexpr int64_t kMaxContainerThreshold = 1000 * kMB;
constexpr int64_t kMaxInt32 = 2147483647;

struct Ctx {
  int nthreads = 1;
  std::string err;
  bool have_nodes = false, have_wl = false, have_prof = false;
  ksg_profile prof{};
  // cluster
  int32_t N = 0, R = 0, L = 0, T = 0, I = 0, V = 0;
  std::vector<int64_t> alloc, requested, nonzero;
  std::vector<int32_t> allowed, pod_count;
  std::vector<uint8_t> unsched;
  std::vector<uint32_t> label_val;
  std::vector<int64_t> label_num;
  std::vector<uint8_t> label_num_ok;
  std::vector<uint32_t> taints;
  std::vector<uint8_t> taint_effect;
  std::vector<uint32_t> images;
  // topology
  std::vector<int32_t> tmpl_col, tmpl_kind, tmpl_weight, col_vocab;
  std::vector<double> log_table;
  // snapshot at load (reset)
  std::vector<int64_t> requested0, nonzero0;
  std::vector<int32_t> pod_count0;
  // workload
  std::vector<ksg_pod> pods;
  std::vector<int32_t> prog;
  // per-node pod lists (NodeInfo.Pods)
  std::vector<std::vector<int32_t>> pods_on;
  // NodeInfo.UsedPorts per node: host-port vocabulary ids (a set, as
  // HostPortInfo is: a pod's removal drops its entries whoever else uses them)
  std::vector<std::set<int32_t>> used_ports;
};

inline uint32_t lv(const Ctx& c, int col, int n) { return c.label_val[(size_t)col * c.N + n]; }

bool sorted_has(const int32_t* v, int n, int32_t x) {
  return std::binary_search(v, v + n, x);
}

// ---- requirement programs (encoder.py grammar) -----------------------------
bool eval_req(const Ctx& c, const int32_t*& w, int n) {
  int col = w[0], op = w[1], nv = w[2];
  const int32_t* vals = w + 3;
  w += 3 + nv;
  if (op == 6) return false;  // Never
  uint32_t v = lv(c, col, n);
  switch (op) {
    case 0: {  // In
      if (!v) return false;
      for (int i = 0; i < nv; i++) if ((uint32_t)vals[i] == v) return true;
      return false;
    }
    case 1: {  // NotIn
      if (!v) return true;
      for (int i = 0; i < nv; i++) if ((uint32_t)vals[i] == v) return false;
      return true;
    }
    case 2: return v != 0;
    case 3: return v == 0;
    case 4:
    case 5: {
      if (!v) return false;
      size_t k = (size_t)col * c.N + n;
      if (!c.label_num_ok[k]) return false;
      int64_t bound = (int64_t)(((uint64_t)(uint32_t)vals[1] << 32) | (uint32_t)vals[0]);
      int64_t x = c.label_num[k];
      return op == 4 ? x > bound : x < bound;
    }
  }
  return false;
}

// one NodeSelectorTerm: all requirements; an empty term matches nothing.
bool eval_term(const Ctx& c, const int32_t*& w, int n) {
  int nr = *w++;
  bool ok = nr > 0;
  for (int i = 0; i < nr; i++) ok = eval_req(c, w, n) && ok;  // consume all
  return ok;
}

// ---- volume plugins (encoder.py Encoder._volume_plan program) --------------
// Decoded once per pod, then checked per node: VolumeRestrictions' RWOP
// conflict, VolumeBinding's reasons (1 node affinity conflict, 2 cannot bind /
// provision, 4 bound PV missing), VolumeZone's zone check.
struct VolTerms { bool all; const int32_t* at; int nt; };   // all: matches every node
struct VolProg {
  bool rwop = false;
  std::vector<std::pair<bool, VolTerms>> bound;   // (pv exists, its node affinity)
  std::vector<std::pair<int, VolTerms>> prov;     // (selected node, allowed topologies; nt < 0: cannot provision)
  int zcols[4] = {-1, -1, -1, -1};
  struct Zone { int col, gcol; std::vector<uint32_t> ids, gids; };
  std::vector<Zone> zones;
};

const int32_t* skip_terms(const int32_t* w, int nt) {
  for (int t = 0; t < nt; t++) {
    int nr = *w++;
    for (int r = 0; r < nr; r++) w += 3 + w[2];
  }
  return w;
}

VolProg decode_vol(const Ctx& c, const ksg_pod& p) {
  VolProg v;
  if (p.vol < 0) return v;
  const int32_t* w = c.prog.data() + p.vol;
  v.rwop = (w[0] & 1) != 0;
  w++;
  int nb = *w++;
  for (int b = 0; b < nb; b++) {
    int kind = *w++;
    if (kind == 0) { v.bound.push_back({false, {true, nullptr, 0}}); continue; }
    int nt = *w++;
    if (nt < 0) { v.bound.push_back({true, {true, nullptr, 0}}); continue; }
    v.bound.push_back({true, {false, w, nt}});
    w = skip_terms(w, nt);
  }
  int np = *w++;
  for (int k = 0; k < np; k++) {
    int sel = *w++, nt = *w++;
    v.prov.push_back({sel, {false, w, nt}});
    if (nt > 0) w = skip_terms(w, nt);
  }
  for (int k = 0; k < 4; k++) v.zcols[k] = *w++;
  int nz = *w++;
  for (int k = 0; k < nz; k++) {
    VolProg::Zone z;
    z.col = w[0];
    z.gcol = w[1];
    int nv = w[2];
    for (int i = 0; i < nv; i++) z.ids.push_back((uint32_t)w[3 + i]);
    int ng = w[3 + nv];
    for (int i = 0; i < ng; i++) z.gids.push_back((uint32_t)w[4 + nv + i]);
    w += 4 + nv + ng;
    v.zones.push_back(std::move(z));
  }
  return v;
}

bool terms_match(const Ctx& c, const VolTerms& t, int n) {
  if (t.all) return true;
  const int32_t* w = t.at;
  bool any = false;
  for (int k = 0; k < t.nt; k++) any = eval_term(c, w, n) || any;
  return any;
}

// FindPodVolumes' reasons at node n: checkBoundClaims stops at the first
// claim whose PV is missing or does not fit; then the unbound claims'
// selected node and provisioning checks
uint32_t volume_binding_reasons(const Ctx& c, const VolProg& v, int n) {
  uint32_t r = 0;
  for (auto& b : v.bound) {
    if (!b.first) { r |= 4u; break; }
    if (!terms_match(c, b.second, n)) { r |= 1u; break; }
  }
  for (auto& pr : v.prov) {
    bool ok = pr.first == -1 || pr.first == n;
    if (pr.second.nt < 0) ok = false;
    else if (pr.second.nt > 0 && !terms_match(c, pr.second, n)) ok = false;
    if (!ok) { r |= 2u; break; }
  }
  return r;
}

bool volume_zone_conflict(const Ctx& c, const VolProg& v, int n) {
  bool constrained = false;
  for (int k = 0; k < 4; k++) constrained = constrained || (v.zcols[k] >= 0 && lv(c, v.zcols[k], n) != 0);
  if (!constrained) return false;
  for (auto& z : v.zones) {
    uint32_t x = lv(c, z.col, n);
    const std::vector<uint32_t>* set = &z.ids;
    if (!x) { x = lv(c, z.gcol, n); set = &z.gids; }
    if (!x || std::find(set->begin(), set->end(), x) == set->end()) return true;
  }
  return false;
}

bool na_required_match(const Ctx& c, const ksg_pod& p, int n) {
  if (p.na_req < 0) return true;
  const int32_t* w = c.prog.data() + p.na_req;
  int nsel = *w++;
  bool ok = true;
  for (int i = 0; i < nsel; i++) ok = eval_req(c, w, n) && ok;
  if (!ok) return false;
  int nterms = *w++;
  if (nterms < 0) return true;
  bool any = false;
  for (int t = 0; t < nterms; t++) any = eval_term(c, w, n) || any;
  return any;
}

int64_t na_pref_score(const Ctx& c, const ksg_pod& p, int n) {
  const int32_t* w = c.prog.data() + p.na_pref;
  int nterms = *w++;
  int64_t s = 0;
  for (int t = 0; t < nterms; t++) {
    int weight = *w++;
    if (eval_term(c, w, n)) s += weight;
  }
  return s;
}

inline bool tol_bit(const Ctx& c, const ksg_pod& p, int which, uint32_t vid) {
  int W = std::max(1, (c.V + 31) / 32);
  const int32_t* b = c.prog.data() + p.tol + which * W;
  return (((uint32_t)b[vid >> 5]) >> (vid & 31)) & 1u;
}

// FindMatchingUntoleratedTaint over NoSchedule|NoExecute; returns slot or -1.
int untolerated_slot(const Ctx& c, const ksg_pod& p, int n) {
  for (int s = 0; s < c.T; s++) {
    uint32_t id = c.taints[(size_t)s * c.N + n];
    if (!id) break;
    uint32_t vid = id - 1;
    uint8_t e = c.taint_effect[vid];
    if (e != KSG_EFFECT_NO_SCHEDULE && e != KSG_EFFECT_NO_EXECUTE) continue;
    if (!tol_bit(c, p, 0, vid)) return s;
  }
  return -1;
}

int64_t taint_score(const Ctx& c, const ksg_pod& p, int n) {
  int64_t k = 0;
  for (int s = 0; s < c.T; s++) {
    uint32_t id = c.taints[(size_t)s * c.N + n];
    if (!id) break;
    uint32_t vid = id - 1;
    if (c.taint_effect[vid] != KSG_EFFECT_PREFER_NO_SCHEDULE) continue;
    if (!tol_bit(c, p, 1, vid)) k++;
  }
  return k;
}

// ---- NodeResourcesFit ------------------------------------------------------
uint32_t fit_filter(const Ctx& c, const ksg_pod& p, int n) {
  uint32_t bits = 0;
  if ((int64_t)c.pod_count[n] + 1 > (int64_t)c.allowed[n]) bits |= 1u;
  for (int r = 0; r < c.R; r++) {
    int64_t q = p.req[r];
    if (q <= 0) continue;  // zero request is never insufficient
    if (r >= 3 && ((c.prof.fit_ignored_res >> r) & 1u)) continue;
    int64_t a = c.alloc[(size_t)r * c.N + n], u = c.requested[(size_t)r * c.N + n];
    if (q > a - u) bits |= 1u << (r + 1);
  }
  return bits;
}

void alloc_req(const Ctx& c, const ksg_pod& p, int r, int n, bool use_requested, int64_t& a, int64_t& q) {
  int64_t pr;
  if (use_requested) pr = p.req[r];
  else pr = r == KSG_RES_CPU ? p.nz_cpu : r == KSG_RES_MEM ? p.nz_mem : p.req[r];
  a = 0; q = 0;
  if (pr == 0 && r >= 3) return;
  a = c.alloc[(size_t)r * c.N + n];
  int64_t base;
  if (!use_requested && r == KSG_RES_CPU) base = c.nonzero[n];
  else if (!use_requested && r == KSG_RES_MEM) base = c.nonzero[(size_t)c.N + n];
  else base = c.requested[(size_t)r * c.N + n];
  q = base + pr;
}

// RequestedToCapacityRatio's broken-line function of utilization u in
// [0, 100] [upstream v1.32 helper/shape_score.go BuildBrokenLinearFunction;
// not vendored, parity unpinned]: left of the first point its score, right of
// the last point the last score, else linear between the two points around u
// (Go int64 division); shape scores arrive already scaled by 100 / 10.
int64_t broken_line(const ksg_profile& pf, int64_t u) {
  int k = 0;
  while (k < pf.shape_n && u > pf.shape_util[k]) k++;
  if (k == pf.shape_n) return pf.shape_score[pf.shape_n - 1];
  if (k == 0) return pf.shape_score[0];
  const int64_t du = pf.shape_util[k] - pf.shape_util[k - 1], ds = pf.shape_score[k] - pf.shape_score[k - 1];
  return pf.shape_score[k - 1] + ds * (u - pf.shape_util[k - 1]) / du;
}

int64_t fit_score(const Ctx& c, const ksg_pod& p, int n) {
  int64_t num = 0, wsum = 0;
  for (int i = 0; i < c.prof.fit_n; i++) {
    int r = c.prof.fit_res[i];
    int64_t a, q;
    alloc_req(c, p, r, n, false, a, q);
    if (a == 0) continue;
    int64_t s;
    if (c.prof.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO) {
      // requested_to_capacity_ratio.go: over capacity scores as full; only
      // resources scoring above zero enter the weighted mean
      s = broken_line(c.prof, q > a ? kMaxNodeScore : q * kMaxNodeScore / a);
      if (s <= 0) continue;
    } else if (c.prof.fit_strategy == KSG_LEAST_ALLOCATED) {
      s = q > a ? 0 : ((a - q) * kMaxNodeScore) / a;
    } else {
      s = ((q > a ? a : q) * kMaxNodeScore) / a;
    }
    num += s * c.prof.fit_w[i];
    wsum += c.prof.fit_w[i];
  }
  if (wsum == 0) return 0;
  if (c.prof.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO)
    return (int64_t)std::round((double)num / (double)wsum);   // math.Round: half away from zero
  return num / wsum;
}

int64_t ba_score(const Ctx& c, const ksg_pod& p, int n) {
  double fr[KSG_MAX_RES];
  int k = 0;
  double total = 0.0;
  for (int i = 0; i < c.prof.ba_n; i++) {
    int64_t a, q;
    alloc_req(c, p, c.prof.ba_res[i], n, true, a, q);
    if (a == 0) continue;
    double f = (double)q / (double)a;
    if (f > 1) f = 1;
    total += f;
    fr[k++] = f;
  }
  double sd = 0.0;
  if (k == 2) {
    sd = std::fabs((fr[0] - fr[1]) / 2);
  } else if (k > 2) {
    double mean = total / (double)k;
    double sum = 0.0;
    for (int i = 0; i < k; i++) sum = sum + (fr[i] - mean) * (fr[i] - mean);
    sd = std::sqrt(sum / (double)k);
  }
  return (int64_t)((1 - sd) * (double)kMaxNodeScore);
}

int64_t image_score(const Ctx& c, const ksg_pod& p, int n) {
  int64_t sum = 0;
  if (p.img >= 0) {
    const int32_t* w = c.prog.data() + p.img;
    int cnt = *w++;
    for (int i = 0; i < cnt; i++, w += 3) {
      uint32_t id = (uint32_t)w[0];
      int64_t contrib = (int64_t)(((uint64_t)(uint32_t)w[2] << 32) | (uint32_t)w[1]);
      for (int s = 0; s < c.I; s++) {
        uint32_t x = c.images[(size_t)s * c.N + n];
        if (!x || x > id) break;
        if (x == id) { sum += contrib; break; }
      }
    }
  }
  int64_t mx = kMaxContainerThreshold * (int64_t)p.n_containers;
  if (sum < kMinThreshold) sum = kMinThreshold;
  else if (sum > mx) sum = mx;
  return kMaxNodeScore * (sum - kMinThreshold) / (mx - kMinThreshold);
}

// ---- selectors / templates -------------------------------------------------
struct CommitProg {
  const int32_t* sels = nullptr; int nsel = 0;
  const int32_t* tmpls = nullptr; int ntmpl = 0;   // ntmpl {template id, weight} pairs
};
CommitProg commit_prog(const Ctx& c, int pod) {
  CommitProg cp;
  int off = c.pods[pod].commit;
  if (off < 0) return cp;
  const int32_t* w = c.prog.data() + off;
  cp.nsel = *w++; cp.sels = w; w += cp.nsel;
  cp.ntmpl = *w++; cp.tmpls = w;
  return cp;
}
bool pod_matches_sel(const Ctx& c, int q, int sel) {
  if (sel < 0) return false;
  CommitProg cp = commit_prog(c, q);
  return sorted_has(cp.sels, cp.nsel, sel);
}
int count_matching(const Ctx& c, int n, int sel) {  // countPodsMatchSelector
  if (sel < 0) return 0;
  int k = 0;
  for (int q : c.pods_on[n]) k += pod_matches_sel(c, q, sel);
  return k;
}

// ---- PodTopologySpread ------------------------------------------------------
struct PtsHard { int col, sel, max_skew, min_domains, self_match, na, nt; };
struct PtsSoft { int col, sel, max_skew, na, nt, hostname; };
struct PtsProg { std::vector<PtsHard> hard; std::vector<PtsSoft> soft; int require_all = 0; };
PtsProg pts_prog(const Ctx& c, const ksg_pod& p) {
  PtsProg g;
  if (p.pts < 0) return g;
  const int32_t* w = c.prog.data() + p.pts;
  int nh = w[0], ns = w[1];
  g.require_all = w[2];
  w += 3;
  for (int i = 0; i < nh; i++, w += 7) g.hard.push_back({w[0], w[1], w[2], w[3], w[4], w[5], w[6]});
  for (int i = 0; i < ns; i++, w += 6) g.soft.push_back({w[0], w[1], w[2], w[3], w[4], w[5]});
  return g;
}
bool inclusion(const Ctx& c, const ksg_pod& p, int na, int nt, int n) {
  if (na && !na_required_match(c, p, n)) return false;
  if (nt && untolerated_slot(c, p, n) >= 0) return false;
  return true;
}

struct PtsPre {  // podtopologyspread preFilterState
  std::vector<std::map<uint32_t, int64_t>> tp;
  std::vector<int64_t> mins;
};
PtsPre pts_prefilter(const Ctx& c, const ksg_pod& p, const PtsProg& g) {
  PtsPre s;
  size_t H = g.hard.size();
  s.tp.resize(H);
  int nth = c.nthreads;
  std::vector<std::vector<std::map<uint32_t, int64_t>>> part(nth, std::vector<std::map<uint32_t, int64_t>>(H));
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int n = 0; n < c.N; n++) {
    bool all = true;
    for (auto& h : g.hard) all = all && lv(c, h.col, n) != 0;
    if (!all) continue;
    auto& mine = part[omp_get_thread_num()];
    for (size_t i = 0; i < H; i++) {
      const PtsHard& h = g.hard[i];
      if (!inclusion(c, p, h.na, h.nt, n)) continue;
      mine[i][lv(c, h.col, n)] += count_matching(c, n, h.sel);
    }
  }
  for (int t = 0; t < nth; t++)
    for (size_t i = 0; i < H; i++)
      for (auto& kv : part[t][i]) s.tp[i][kv.first] += kv.second;
  for (size_t i = 0; i < H; i++) {
    int64_t mn = kMaxInt32;
    for (auto& kv : s.tp[i]) mn = std::min(mn, kv.second);
    if ((int64_t)s.tp[i].size() < g.hard[i].min_domains) mn = 0;
    s.mins.push_back(mn);
  }
  return s;
}
uint32_t pts_filter(const Ctx& c, const PtsProg& g, const PtsPre& s, int n) {
  for (size_t i = 0; i < g.hard.size(); i++) {
    const PtsHard& h = g.hard[i];
    uint32_t v = lv(c, h.col, n);
    if (!v) return 1;
    auto it = s.tp[i].find(v);
    int64_t cnt = it == s.tp[i].end() ? 0 : it->second;
    if (cnt + h.self_match - s.mins[i] > h.max_skew) return 2;
  }
  return 0;
}

struct PtsScore {
  std::vector<uint8_t> ignored;  // per node
  std::vector<std::map<uint32_t, int64_t>> counts;
  std::vector<double> weight;
};
inline uint32_t dom_or_empty(const Ctx& c, int col, int n) {
  uint32_t v = lv(c, col, n);
  return v ? v : 1u;  // node.Labels[key] of a missing key is "" (value id 1)
}
bool has_all_soft(const Ctx& c, const PtsProg& g, int n) {
  for (auto& s : g.soft) if (!lv(c, s.col, n)) return false;
  return true;
}
PtsScore pts_prescore(const Ctx& c, const ksg_pod& p, const PtsProg& g, const std::vector<int>& feas) {
  PtsScore st;
  size_t S = g.soft.size();
  st.ignored.assign(c.N, 0);
  st.counts.resize(S);
  std::vector<int64_t> topo(S, 0);
  int64_t n_ignored = 0;
  for (int n : feas) {
    if (g.require_all && !has_all_soft(c, g, n)) { st.ignored[n] = 1; n_ignored++; continue; }
    for (size_t i = 0; i < S; i++) {
      if (g.soft[i].hostname) continue;
      uint32_t v = dom_or_empty(c, g.soft[i].col, n);
      if (!st.counts[i].count(v)) { st.counts[i][v] = 0; topo[i]++; }
    }
  }
  for (size_t i = 0; i < S; i++) {
    int64_t sz = topo[i];
    if (g.soft[i].hostname) sz = (int64_t)feas.size() - n_ignored;
    st.weight.push_back(c.log_table[sz + 2]);
  }
  int nth = c.nthreads;
  std::vector<std::vector<std::map<uint32_t, int64_t>>> part(nth, std::vector<std::map<uint32_t, int64_t>>(S));
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int n = 0; n < c.N; n++) {
    if (g.require_all && !has_all_soft(c, g, n)) continue;
    auto& mine = part[omp_get_thread_num()];
    for (size_t i = 0; i < S; i++) {
      const PtsSoft& s = g.soft[i];
      if (!inclusion(c, p, s.na, s.nt, n)) continue;
      uint32_t v = dom_or_empty(c, s.col, n);
      if (!st.counts[i].count(v)) continue;
      mine[i][v] += count_matching(c, n, s.sel);
    }
  }
  for (int t = 0; t < nth; t++)
    for (size_t i = 0; i < S; i++)
      for (auto& kv : part[t][i]) st.counts[i][kv.first] += kv.second;
  return st;
}
int64_t pts_score(const Ctx& c, const PtsProg& g, const PtsScore& st, int n) {
  if (st.ignored[n]) return 0;
  double score = 0.0;
  for (size_t i = 0; i < g.soft.size(); i++) {
    const PtsSoft& s = g.soft[i];
    uint32_t v = lv(c, s.col, n);
    if (!v) continue;
    int64_t cnt;
    if (s.hostname) cnt = count_matching(c, n, s.sel);
    else cnt = st.counts[i].at(v);
    double t = (double)cnt * st.weight[i];
    score += t + (double)(s.max_skew - 1);
  }
  return (int64_t)std::round(score);
}

// ---- InterPodAffinity --------------------------------------------------------
struct IpaProg {
  int n_aff = 0, sel_all = -1, self_all = 0;
  std::vector<int> aff_cols;
  std::vector<std::pair<int, int>> anti;           // (col, sel)
  struct Pref { int col, sel, w; };
  std::vector<Pref> pref;
  std::vector<int32_t> m_anti, m_hard, m_pref;     // sorted template ids
};
IpaProg ipa_prog(const Ctx& c, const ksg_pod& p) {
  IpaProg g;
  if (p.ipa < 0) return g;
  const int32_t* w = c.prog.data() + p.ipa;
  g.n_aff = w[0]; g.sel_all = w[1]; g.self_all = w[2]; w += 3;
  for (int i = 0; i < g.n_aff; i++) g.aff_cols.push_back(*w++);
  int na = *w++;
  for (int i = 0; i < na; i++, w += 2) g.anti.push_back({w[0], w[1]});
  int np = *w++;
  for (int i = 0; i < np; i++, w += 3) g.pref.push_back({w[0], w[1], w[2]});
  for (auto* v : {&g.m_anti, &g.m_hard, &g.m_pref}) {
    int k = *w++;
    v->assign(w, w + k);
    w += k;
    std::sort(v->begin(), v->end());
  }
  return g;
}
using PairMap = std::map<std::pair<int, uint32_t>, int64_t>;
struct IpaPre { PairMap existing_anti, aff, anti; bool skip = false; };

IpaPre ipa_prefilter(const Ctx& c, const ksg_pod& p, const IpaProg& g) {
  IpaPre s;
  int nth = c.nthreads;
  std::vector<PairMap> pe(nth), pa(nth), pn(nth);
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int n = 0; n < c.N; n++) {
    int t = omp_get_thread_num();
    for (int q : c.pods_on[n]) {
      CommitProg cp = commit_prog(c, q);
      for (int k = 0; k < cp.ntmpl; k++) {
        int tid = cp.tmpls[2 * k];
        if (c.tmpl_kind[tid] != KSG_TMPL_REQ_ANTI) continue;
        if (!std::binary_search(g.m_anti.begin(), g.m_anti.end(), tid)) continue;
        uint32_t v = lv(c, c.tmpl_col[tid], n);
        if (v) pe[t][{c.tmpl_col[tid], v}] += 1;
      }
      if (g.n_aff > 0 && sorted_has(cp.sels, cp.nsel, g.sel_all))
        for (int col : g.aff_cols) {
          uint32_t v = lv(c, col, n);
          if (v) pa[t][{col, v}] += 1;
        }
      for (auto& a : g.anti)
        if (sorted_has(cp.sels, cp.nsel, a.second)) {
          uint32_t v = lv(c, a.first, n);
          if (v) pn[t][{a.first, v}] += 1;
        }
    }
  }
  for (int t = 0; t < nth; t++) {
    for (auto& kv : pe[t]) s.existing_anti[kv.first] += kv.second;
    for (auto& kv : pa[t]) s.aff[kv.first] += kv.second;
    for (auto& kv : pn[t]) s.anti[kv.first] += kv.second;
  }
  s.skip = s.existing_anti.empty() && g.n_aff == 0 && g.anti.empty();
  return s;
}
uint32_t ipa_filter(const Ctx& c, const IpaProg& g, const IpaPre& s, int n) {
  bool pods_exist = true;
  for (int col : g.aff_cols) {
    uint32_t v = lv(c, col, n);
    if (!v) return 1;
    auto it = s.aff.find({col, v});
    if (it == s.aff.end() || it->second <= 0) pods_exist = false;
  }
  if (!pods_exist && !(s.aff.empty() && g.n_aff > 0 && g.self_all)) return 1;
  if (!s.anti.empty())
    for (auto& a : g.anti) {
      uint32_t v = lv(c, a.first, n);
      if (!v) continue;
      auto it = s.anti.find({a.first, v});
      if (it != s.anti.end() && it->second > 0) return 2;
    }
  for (auto& kv : s.existing_anti)
    if (kv.second > 0 && lv(c, kv.first.first, n) == kv.first.second) return 3;
  return 0;
}
struct IpaScore { PairMap topo; bool empty = true; };
IpaScore ipa_prescore(const Ctx& c, const ksg_pod& p, const IpaProg& g) {
  IpaScore st;
  bool has_cons = !g.pref.empty();
  int64_t hw = c.prof.hard_pod_affinity_weight;
  int nth = c.nthreads;
  std::vector<PairMap> part(nth);
  std::vector<uint8_t> any(nth, 0);
#pragma omp parallel for num_threads(nth) schedule(static)
  for (int n = 0; n < c.N; n++) {
    int t = omp_get_thread_num();
    for (int q : c.pods_on[n]) {
      CommitProg cp = commit_prog(c, q);
      if (!has_cons && cp.ntmpl == 0) continue;  // only pods with affinity
      for (auto& pr : g.pref)
        if (sorted_has(cp.sels, cp.nsel, pr.sel)) {
          uint32_t v = lv(c, pr.col, n);
          if (v) { part[t][{pr.col, v}] += pr.w; any[t] = 1; }
        }
      for (int k = 0; k < cp.ntmpl; k++) {
        int tid = cp.tmpls[2 * k];
        int kind = c.tmpl_kind[tid];
        int64_t add;
        if (kind == KSG_TMPL_REQ_AFF) {
          if (hw <= 0 || !std::binary_search(g.m_hard.begin(), g.m_hard.end(), tid)) continue;
          add = hw;
        } else if (kind == KSG_TMPL_PREF) {
          if (!std::binary_search(g.m_pref.begin(), g.m_pref.end(), tid)) continue;
          add = cp.tmpls[2 * k + 1];   // the owning term's signed weight
        } else {
          continue;
        }
        uint32_t v = lv(c, c.tmpl_col[tid], n);
        if (v) { part[t][{c.tmpl_col[tid], v}] += add; any[t] = 1; }
      }
    }
  }
  for (int t = 0; t < nth; t++) {
    for (auto& kv : part[t]) st.topo[kv.first] += kv.second;
    if (any[t]) st.empty = false;
  }
  return st;
}
int64_t ipa_score(const Ctx& c, const IpaScore& st, int n) {
  int64_t s = 0;
  for (auto& kv : st.topo)
    if (lv(c, kv.first.first, n) == kv.first.second) s += kv.second;
  return s;
}

// ---- one scheduling cycle ----------------------------------------------------
bool in_filter(const Ctx& c, int pl) {
  for (int k = 0; k < c.prof.n_filter; k++) if (c.prof.filter_order[k] == pl) return true;
  return false;
}

int eval_pod(Ctx& c, int pi, ksg_result* res, ksg_capture* cap) {
  const ksg_pod& p = c.pods[pi];
  const int N = c.N;
  res->selected = -1;
  res->n_feasible = 0;
  res->status = 0;
  res->score_skip = p.score_skip;
  std::vector<uint32_t> fs(N, KSG_FS_NOT_EVALUATED);
  // InterPodAffinity's PreFilter Skip is reported for every pod, a pod that
  // another PreFilter rejected included (the status bit then matters only
  // when InterPodAffinity precedes the rejecting plugin in PreFilter order)
  IpaProg ig = ipa_prog(c, p);
  IpaPre ipre;
  ipre.skip = true;
  if (p.ipa >= 0 && in_filter(c, KSG_PL_INTER_POD_AFFINITY)) ipre = ipa_prefilter(c, p, ig);
  if (ipre.skip && in_filter(c, KSG_PL_INTER_POD_AFFINITY)) res->status |= KSG_ST_IPA_PREFILTER_SKIP;
  if (!(p.flags & KSG_POD_PREFILTER_REJECT)) {
    uint32_t fskip = p.filter_skip;
    PtsProg pg = pts_prog(c, p);
    PtsPre pre;
    if (!((fskip >> KSG_PL_POD_TOPOLOGY_SPREAD) & 1) && in_filter(c, KSG_PL_POD_TOPOLOGY_SPREAD))
      pre = pts_prefilter(c, p, pg);
    if (ipre.skip) fskip |= 1u << KSG_PL_INTER_POD_AFFINITY;
    const int32_t* node_set = p.node_set >= 0 ? c.prog.data() + p.node_set : nullptr;
    const VolProg vp = decode_vol(c, p);
#pragma omp parallel for num_threads(c.nthreads) schedule(static)
    for (int n = 0; n < N; n++) {
      if (node_set && !((((uint32_t)node_set[n >> 5]) >> (n & 31)) & 1u)) continue;
      uint32_t st = 0;
      for (int k = 0; k < c.prof.n_filter && !st; k++) {
        int pl = c.prof.filter_order[k];
        if ((fskip >> pl) & 1u) continue;
        uint32_t reason = 0;
        bool fail = false;
        switch (pl) {
          case KSG_PL_NODE_UNSCHEDULABLE:
            fail = c.unsched[n] && !(p.flags & KSG_POD_TOL_UNSCHED);
            break;
          case KSG_PL_NODE_NAME:
            fail = p.node_name != -1 && p.node_name != n;
            break;
          case KSG_PL_TAINT_TOLERATION: {
            int s = untolerated_slot(c, p, n);
            if (s >= 0) { fail = true; reason = (uint32_t)s; }
            break;
          }
          case KSG_PL_NODE_AFFINITY:
            if (!na_required_match(c, p, n)) { fail = true; reason = 1; }
            break;
          case KSG_PL_NODE_PORTS:   // nodeports.fitsPorts over the conflict ids (encoder.py ports grammar)
            if (p.ports >= 0) {
              const int32_t* w = c.prog.data() + p.ports;
              for (int i = 0; i < w[0] && !fail; i++) fail = c.used_ports[n].count(w[1 + i]) != 0;
            }
            break;
          case KSG_PL_NODE_RESOURCES_FIT: {
            uint32_t b = fit_filter(c, p, n);
            if (b) { fail = true; reason = b; }
            break;
          }
          case KSG_PL_POD_TOPOLOGY_SPREAD: {
            uint32_t r = pts_filter(c, pg, pre, n);
            if (r) { fail = true; reason = r; }
            break;
          }
          case KSG_PL_INTER_POD_AFFINITY: {
            uint32_t r = ipa_filter(c, ig, ipre, n);
            if (r) { fail = true; reason = r; }
            break;
          }
          case KSG_PL_VOLUME_RESTRICTIONS:
            fail = vp.rwop;
            break;
          case KSG_PL_VOLUME_BINDING: {
            uint32_t r = p.vol >= 0 ? volume_binding_reasons(c, vp, n) : 0;
            if (r) { fail = true; reason = r; }
            break;
          }
          case KSG_PL_VOLUME_ZONE:
            fail = p.vol >= 0 && volume_zone_conflict(c, vp, n);
            break;
          default:
            break;  // NodeVolumeLimits: passes (no CSI attach limits modelled)
        }
        if (fail) st = (uint32_t)(pl + 1) | (reason << 8);
      }
      fs[n] = st;
    }
  }
  std::vector<int> feas;
  for (int n = 0; n < N; n++) if (fs[n] == 0) feas.push_back(n);
  res->n_feasible = (int32_t)feas.size();
  if (cap && cap->fstatus) std::memcpy(cap->fstatus, fs.data(), sizeof(uint32_t) * N);
  if (feas.empty()) return KSG_OK;
  if (feas.size() == 1) { res->selected = feas[0]; return KSG_OK; }
  res->status |= KSG_ST_SCORED;

  // PreScore
  uint32_t sskip = p.score_skip;
  PtsProg pg = pts_prog(c, p);
  PtsScore pst;
  if (!((sskip >> KSG_PL_POD_TOPOLOGY_SPREAD) & 1u) && (c.prof.score_mask >> KSG_PL_POD_TOPOLOGY_SPREAD & 1u))
    pst = pts_prescore(c, p, pg, feas);
  IpaScore ist;
  if ((c.prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) {
    if (!((sskip >> KSG_PL_INTER_POD_AFFINITY) & 1u)) {
      if (p.ipa >= 0) ist = ipa_prescore(c, p, ig);
      if (ist.empty) { sskip |= 1u << KSG_PL_INTER_POD_AFFINITY; res->status |= KSG_ST_IPA_PRESCORE_SKIP; }
    }
  }
  res->score_skip = sskip;

  const size_t F = feas.size();
  std::vector<int64_t> total(F, 0);
  std::vector<int64_t> raw(F), norm(F);
  // RunScorePlugins: Score() of every plugin for every feasible node (one
  // parallel pass over nodes, like the upstream Parallelizer), then
  // NormalizeScore per plugin.
  int plugins[KSG_NPLUGINS], np = 0;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    if (((c.prof.score_mask >> pl) & 1u) && !((sskip >> pl) & 1u)) plugins[np++] = pl;
  std::vector<int64_t> rawm((size_t)np * F);
#pragma omp parallel for num_threads(c.nthreads) schedule(static)
  for (size_t i = 0; i < F; i++) {
    const int n = feas[i];
    for (int k = 0; k < np; k++) {
      int64_t s = 0;
      switch (plugins[k]) {
        case KSG_PL_NODE_RESOURCES_FIT: s = fit_score(c, p, n); break;
        case KSG_PL_BALANCED_ALLOCATION: s = ba_score(c, p, n); break;
        case KSG_PL_TAINT_TOLERATION: s = taint_score(c, p, n); break;
        case KSG_PL_NODE_AFFINITY: s = na_pref_score(c, p, n); break;
        case KSG_PL_IMAGE_LOCALITY: s = image_score(c, p, n); break;
        case KSG_PL_POD_TOPOLOGY_SPREAD: s = pts_score(c, pg, pst, n); break;
        case KSG_PL_INTER_POD_AFFINITY: s = ipa_score(c, ist, n); break;
        default: s = 0; break;
      }
      rawm[(size_t)k * F + i] = s;
    }
  }
  // NormalizeScore statistics per plugin (serial, no division) ...
  int64_t s_min[KSG_NPLUGINS], s_max[KSG_NPLUGINS];
  for (int k = 0; k < np; k++) {
    const int pl = plugins[k];
    const int64_t* r = rawm.data() + (size_t)k * F;
    int64_t mn = INT64_MAX, mx = pl == KSG_PL_INTER_POD_AFFINITY ? INT64_MIN : 0;
    for (size_t i = 0; i < F; i++) {
      if (pl == KSG_PL_POD_TOPOLOGY_SPREAD && pst.ignored[feas[i]]) continue;
      mn = std::min(mn, r[i]);
      mx = std::max(mx, r[i]);
    }
    s_min[k] = mn;
    s_max[k] = mx;
  }
  // ... then normalise, weight and sum per node (parallel).
  uint32_t err = 0;
#pragma omp parallel for num_threads(c.nthreads) schedule(static) reduction(| : err)
  for (size_t i = 0; i < F; i++) {
    int64_t t = 0;
    for (int k = 0; k < np; k++) {
      const int pl = plugins[k];
      const int64_t x = rawm[(size_t)k * F + i], mn = s_min[k], mx = s_max[k];
      int64_t v = x;
      if (pl == KSG_PL_TAINT_TOLERATION || pl == KSG_PL_NODE_AFFINITY) {
        // helper.DefaultNormalizeScore(MaxNodeScore, reverse)
        const bool reverse = pl == KSG_PL_TAINT_TOLERATION;
        if (mx == 0) v = reverse ? kMaxNodeScore : x;
        else {
          const int64_t sc = kMaxNodeScore * x / mx;
          v = reverse ? kMaxNodeScore - sc : sc;
        }
      } else if (pl == KSG_PL_POD_TOPOLOGY_SPREAD) {
        if (pst.ignored[feas[i]]) v = 0;
        else if (mx == 0) v = kMaxNodeScore;
        else v = kMaxNodeScore * (mx + mn - x) / mx;
      } else if (pl == KSG_PL_INTER_POD_AFFINITY) {
        const int64_t diff = mx - mn;
        double f = 0;
        if (diff > 0) f = (double)kMaxNodeScore * ((double)(x - mn) / (double)diff);
        v = (int64_t)f;
      }
      if (v > kMaxNodeScore || v < 0) err |= 1u;
      t += v * c.prof.weight[pl];
      if (cap && cap->raw) {
        cap->raw[(size_t)pl * N + feas[i]] = x;
        cap->norm[(size_t)pl * N + feas[i]] = v;
      }
    }
    total[i] = t;
  }
  if (err) res->status |= KSG_ST_SCORE_ERROR;
  if (res->status & KSG_ST_SCORE_ERROR) return KSG_OK;  // framework error: no placement
  size_t best = 0;
  for (size_t i = 1; i < F; i++)
    if (total[i] > total[best]) best = i;  // ties: lowest node index (feas ascending)
  res->selected = feas[best];
  if (cap && cap->total)
    for (size_t i = 0; i < F; i++) cap->total[feas[i]] = total[i];
  return KSG_OK;
}

void commit(Ctx& c, int pi, int n) {
  const ksg_pod& p = c.pods[pi];
  for (int r = 0; r < c.R; r++) c.requested[(size_t)r * c.N + n] += p.req[r];
  c.nonzero[n] += p.nz_cpu;
  c.nonzero[(size_t)c.N + n] += p.nz_mem;
  c.pod_count[n] += 1;
  c.pods_on[n].push_back(pi);
  if (p.ports >= 0) {   // UsedPorts.Add of the pod's own ids
    const int32_t* own = c.prog.data() + p.ports + 1 + c.prog[p.ports];
    for (int i = 0; i < own[0]; i++) c.used_ports[n].insert(own[1 + i]);
  }
}

// NodeInfo.RemovePod for a preemption victim (the inverse of commit).
void uncommit(Ctx& c, int pi, int n) {
  const ksg_pod& p = c.pods[pi];
  for (int r = 0; r < c.R; r++) c.requested[(size_t)r * c.N + n] -= p.req[r];
  c.nonzero[n] -= p.nz_cpu;
  c.nonzero[(size_t)c.N + n] -= p.nz_mem;
  c.pod_count[n] -= 1;
  auto& v = c.pods_on[n];
  v.erase(std::find(v.begin(), v.end(), pi));
  if (p.ports >= 0) {   // UsedPorts.Remove
    const int32_t* own = c.prog.data() + p.ports + 1 + c.prog[p.ports];
    for (int i = 0; i < own[0]; i++) c.used_ports[n].erase(own[1 + i]);
  }
}

// defaultpreemption.SelectVictimsOnNode (upstream v1.32): on the node, remove
// every lower-priority pod, run the filters, reprieve the pods most important
// first.  Upstream keeps the cloned PreFilter state in step with each removal
// and re-addition through the plugins' RemovePod / AddPod extensions; here the
// PodTopologySpread and InterPodAffinity PreFilter states are recomputed from
// scratch on the modified cluster (the same counts, by their definition), with
// the PreFilter Skip decisions of the original cycle; NodePorts reads the
// node's UsedPorts as the removals leave them.  The node's pods are restored
// afterwards.  Node-static filters are not re-run: the caller only passes
// nodes whose first rejection came from Fit / NodePorts / PTS / IPA with every
// static filter ordered before them (preemption.check_scope).
void select_victims(Ctx& c, int pi, int n, const int32_t* vic, int nv, int32_t& fits, uint8_t* victim) {
  const ksg_pod& p = c.pods[pi];
  const uint32_t fskip = p.filter_skip;
  auto on = [&](int pl) { return in_filter(c, pl) && !((fskip >> pl) & 1u); };
  const bool fit_on = on(KSG_PL_NODE_RESOURCES_FIT);
  const PtsProg pg = pts_prog(c, p);
  const bool pts_on = on(KSG_PL_POD_TOPOLOGY_SPREAD) && !pg.hard.empty();
  const IpaProg ig = ipa_prog(c, p);
  bool ipa_on = false;
  if (p.ipa >= 0 && on(KSG_PL_INTER_POD_AFFINITY)) ipa_on = !ipa_prefilter(c, p, ig).skip;
  // NodePorts on the node's UsedPorts as the removals / re-additions leave
  // them (uncommit / commit: set semantics, upstream HostPortInfo)
  const bool ports_on = on(KSG_PL_NODE_PORTS) && p.ports >= 0;
  auto passes = [&]() {
    if (ports_on) {
      const int32_t* w = c.prog.data() + p.ports;
      for (int i = 0; i < w[0]; i++)
        if (c.used_ports[n].count(w[1 + i])) return false;
    }
    if (fit_on && fit_filter(c, p, n) != 0) return false;
    if (pts_on && pts_filter(c, pg, pts_prefilter(c, p, pg), n) != 0) return false;
    if (ipa_on && ipa_filter(c, ig, ipa_prefilter(c, p, ig), n) != 0) return false;
    return true;
  };
  std::vector<int> removed;
  for (int i = 0; i < nv; i++) { uncommit(c, vic[i], n); removed.push_back(vic[i]); }
  fits = passes() ? 1 : 0;
  for (int i = 0; i < nv; i++) {
    victim[i] = 0;
    if (!fits) continue;
    commit(c, vic[i], n);                          // reprievePod
    removed.erase(std::find(removed.begin(), removed.end(), vic[i]));
    if (!passes()) {
      uncommit(c, vic[i], n);
      removed.push_back(vic[i]);
      victim[i] = 1;
    }
  }
  for (int q : removed) commit(c, q, n);
}

}  // namespace

struct kso_ctx : Ctx {};

extern "C" {

int kso_open(int nthreads, kso_ctx** out) {
  if (!out) return KSG_E_INVALID;
  kso_ctx* c = new kso_ctx();
  c->nthreads = nthreads > 0 ? nthreads : 1;
  *out = c;
  return KSG_OK;
}
int kso_close(kso_ctx* c) { delete c; return KSG_OK; }
const char* kso_last_error(kso_ctx* c) { return c ? c->err.c_str() : "null ctx"; }
int kso_set_threads(kso_ctx* c, int nthreads) { c->nthreads = nthreads > 0 ? nthreads : 1; return KSG_OK; }

int kso_set_profile(kso_ctx* c, const ksg_profile* p) {
  if (!c || !p) return KSG_E_INVALID;
  c->prof = *p;
  c->have_prof = true;
  return KSG_OK;
}

int kso_load_nodes(kso_ctx* c, const ksg_nodes* nd, const ksg_topology* tp) {
  if (!c || !nd || !tp) return KSG_E_INVALID;
  int N = nd->n_nodes;
  c->N = N; c->R = nd->n_res; c->L = nd->n_label_cols; c->T = nd->max_taints;
  c->I = nd->max_images; c->V = nd->n_taint_vocab;
  auto cp = [](auto& dst, const auto* src, size_t n) { dst.assign(src, src + n); };
  cp(c->alloc, nd->alloc, (size_t)c->R * N);
  cp(c->requested, nd->requested, (size_t)c->R * N);
  cp(c->nonzero, nd->nonzero, (size_t)2 * N);
  cp(c->allowed, nd->allowed_pods, N);
  cp(c->pod_count, nd->pod_count, N);
  cp(c->unsched, nd->unschedulable, N);
  size_t LN = (size_t)std::max(c->L, 1) * N;
  cp(c->label_val, nd->label_val, LN);
  cp(c->label_num, nd->label_num, LN);
  cp(c->label_num_ok, nd->label_num_ok, LN);
  cp(c->taints, nd->taints, (size_t)c->T * N);
  cp(c->taint_effect, nd->taint_effect, (size_t)std::max(c->V, 1));
  cp(c->images, nd->images, (size_t)c->I * N);
  int nt = std::max(tp->n_templates, 1);
  cp(c->tmpl_col, tp->tmpl_col, nt);
  cp(c->tmpl_kind, tp->tmpl_kind, nt);
  cp(c->tmpl_weight, tp->tmpl_weight, nt);
  cp(c->col_vocab, tp->col_vocab, std::max(c->L, 1));
  cp(c->log_table, tp->log_table, tp->log_n);
  c->requested0 = c->requested; c->nonzero0 = c->nonzero; c->pod_count0 = c->pod_count;
  c->pods_on.assign(N, {});
  c->used_ports.assign(N, {});
  c->have_nodes = true;
  return KSG_OK;
}

int kso_load_workload(kso_ctx* c, const ksg_workload* wl) {
  if (!c || !wl) return KSG_E_INVALID;
  c->pods.assign(wl->pods, wl->pods + wl->n_pods);
  c->prog.assign(wl->prog, wl->prog + wl->prog_len);
  c->have_wl = true;
  return KSG_OK;
}

int kso_append_pods(kso_ctx* c, const ksg_workload* tail, int64_t prog_base) {
  if (!c || !tail || !c->have_wl || prog_base < 0 || prog_base > (int64_t)c->prog.size()) return KSG_E_INVALID;
  c->prog.resize(prog_base);
  c->prog.insert(c->prog.end(), tail->prog, tail->prog + tail->prog_len);
  c->pods.insert(c->pods.end(), tail->pods, tail->pods + tail->n_pods);
  return KSG_OK;
}

int kso_eval_pod(kso_ctx* c, const ksg_pod* pod, const int32_t* prog, int64_t prog_len, ksg_result* res,
                 ksg_capture* cap) {
  if (!c || !pod || !res || !c->have_nodes || !c->have_wl || !c->have_prof) return KSG_E_STATE;
  const int64_t base = (int64_t)c->prog.size();
  ksg_pod p = *pod;
  for (int32_t* f : {&p.tol, &p.na_req, &p.na_pref, &p.img, &p.node_set, &p.pts, &p.ipa, &p.commit, &p.blob,
                     &p.ports, &p.vol})
    if (*f >= 0) *f = (int32_t)(*f + base);
  c->prog.insert(c->prog.end(), prog, prog + prog_len);
  c->pods.push_back(p);
  const int rc = eval_pod(*c, (int)c->pods.size() - 1, res, cap);
  c->pods.pop_back();
  c->prog.resize(base);
  return rc;
}

int kso_reset_state(kso_ctx* c) {
  c->requested = c->requested0; c->nonzero = c->nonzero0; c->pod_count = c->pod_count0;
  c->pods_on.assign(c->N, {});
  c->used_ports.assign(c->N, {});
  return KSG_OK;
}

int kso_eval(kso_ctx* c, int32_t pod, ksg_result* res, ksg_capture* cap) {
  if (!c || !res || !c->have_nodes || !c->have_wl || !c->have_prof) return KSG_E_STATE;
  if (pod < 0 || pod >= (int)c->pods.size()) return KSG_E_INVALID;
  return eval_pod(*c, pod, res, cap);
}

// ksg_eval_skipping: the Filter plugins in filter_skip skipped for this call
int kso_eval_skipping(kso_ctx* c, int32_t pod, uint32_t filter_skip, ksg_result* res, ksg_capture* cap) {
  if (!c || !res || !c->have_nodes || !c->have_wl || !c->have_prof) return KSG_E_STATE;
  if (pod < 0 || pod >= (int)c->pods.size()) return KSG_E_INVALID;
  const uint32_t keep = c->pods[pod].filter_skip;
  c->pods[pod].filter_skip |= filter_skip;
  const int rc = eval_pod(*c, pod, res, cap);
  c->pods[pod].filter_skip = keep;
  return rc;
}

int kso_commit(kso_ctx* c, int32_t pod, int32_t node) {
  if (!c || pod < 0 || pod >= (int)c->pods.size() || node < 0 || node >= c->N) return KSG_E_INVALID;
  commit(*c, pod, node);
  return KSG_OK;
}

int kso_uncommit(kso_ctx* c, int32_t pod, int32_t node) {
  if (!c || pod < 0 || pod >= (int)c->pods.size() || node < 0 || node >= c->N) return KSG_E_INVALID;
  auto& v = c->pods_on[node];
  if (std::find(v.begin(), v.end(), pod) == v.end()) { c->err = "uncommit: pod not on node"; return KSG_E_INVALID; }
  uncommit(*c, pod, node);
  return KSG_OK;
}

int kso_preempt_victims(kso_ctx* c, int32_t pod, const int32_t* cand_node, int32_t n_cand, const int32_t* vic_off,
                        const int32_t* vic_pod, int32_t* fits, uint8_t* victim) {
  if (!c || !c->have_nodes || !c->have_wl || !c->have_prof) return KSG_E_STATE;
  if (pod < 0 || pod >= (int)c->pods.size() || n_cand < 0) return KSG_E_INVALID;
  for (int k = 0; k < n_cand; k++) {
    const int n = cand_node[k];
    if (n < 0 || n >= c->N) return KSG_E_INVALID;
    select_victims(*c, pod, n, vic_pod + vic_off[k], vic_off[k + 1] - vic_off[k], fits[k], victim + vic_off[k]);
  }
  return KSG_OK;
}

int kso_run_queue(kso_ctx* c, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                  ksg_capture* cap) {
  if (!c || !c->have_nodes || !c->have_wl || !c->have_prof) return KSG_E_STATE;
  if (first < 0 || count < 0 || first + count > (int)c->pods.size()) return KSG_E_INVALID;
  size_t N = c->N;
  for (int k = 0; k < count; k++) {
    ksg_result r;
    ksg_capture ck, *cp = nullptr;
    if (cap) {
      ck.fstatus = cap->fstatus ? cap->fstatus + (size_t)k * N : nullptr;
      ck.raw = cap->raw ? cap->raw + (size_t)k * KSG_NPLUGINS * N : nullptr;
      ck.norm = cap->norm ? cap->norm + (size_t)k * KSG_NPLUGINS * N : nullptr;
      ck.total = cap->total ? cap->total + (size_t)k * N : nullptr;
      cp = &ck;
    }
    int rc = eval_pod(*c, first + k, &r, cp);
    if (rc) return rc;
    if (r.selected >= 0) commit(*c, first + k, r.selected);
    if (placements) placements[k] = r.selected;
    if (results) results[k] = r;
  }
  return KSG_OK;
}

int kso_read_state(kso_ctx* c, ksg_node_state* out) {
  if (!c || !out) return KSG_E_INVALID;
  std::memcpy(out->requested, c->requested.data(), c->requested.size() * 8);
  std::memcpy(out->nonzero, c->nonzero.data(), c->nonzero.size() * 8);
  std::memcpy(out->pod_count, c->pod_count.data(), c->pod_count.size() * 4);
  return KSG_OK;
}

}  // extern "C"
