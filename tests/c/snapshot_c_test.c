/*
 * snapshot_c_test.c — the drop-in boundary exercised from C only: clusters are
 * built from strings through include/ksched_snapshot.h (no Python encoder),
 * encoded by libksched.so, and scheduled
 *   --cpu : on the C++ oracle only (liboracle.so; test infrastructure):
 *           README KAT scores, incremental-vs-full encoding bytes, oracle
 *           placements of both encodings equal;
 *   --gpu : on the MI355X through ksg_run_queue (whole queue) and through the
 *           per-cycle path a cgo shim takes (add_pod -> sync -> ksg_eval ->
 *           status words -> ksg_snapshot_assume), each compared with the
 *           oracle's placements, results and per-node filter status words.
 * Built by __graft_entry__.build() (gcc, links libksched.so + liboracle.so);
 * run by tests/test_snapshot_c.py.  Exit 0 = every check passed.
 */
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ksched_snapshot.h"

/* ---- the CPU oracle's C ABI (oracle/oracle.cpp; the checker) ---- */
typedef struct kso_ctx kso_ctx;
int kso_open(int nthreads, kso_ctx** out);
int kso_close(kso_ctx* c);
int kso_set_profile(kso_ctx* c, const ksg_profile* p);
int kso_load_nodes(kso_ctx* c, const ksg_nodes* nd, const ksg_topology* tp);
int kso_load_workload(kso_ctx* c, const ksg_workload* wl);
int kso_append_pods(kso_ctx* c, const ksg_workload* tail, int64_t prog_base);
int kso_eval(kso_ctx* c, int32_t pod, ksg_result* res, ksg_capture* cap);
int kso_commit(kso_ctx* c, int32_t pod, int32_t node);
int kso_run_queue(kso_ctx* c, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                  ksg_capture* cap);

static int g_fail = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
      g_fail++;                                           \
    }                                                     \
  } while (0)
#define OK(call)                                                                  \
  do {                                                                            \
    int _rc = (call);                                                             \
    if (_rc != 0) {                                                               \
      fprintf(stderr, "FATAL %s:%d: %s -> %d\n", __FILE__, __LINE__, #call, _rc); \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

/* ---- tiny arena: every string / array lives until exit ---- */
static const char* S(const char* f, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return strdup(buf);
}
static void* A(size_t n, size_t sz) { return calloc(n ? n : 1, sz); }

static uint64_t g_rng = 88172645463325252ull;
static uint32_t rnd(uint32_t n) {   /* xorshift64 */
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (uint32_t)(g_rng % n);
}

#define GI (1024ll * 1024 * 1024)
#define MI (1024ll * 1024)

/* ---- scenario = nodes + pods + bindings + profile ---- */
typedef struct {
  const char* name;
  ksg_profile_view prof;
  int n_nodes, n_pods, n_bound;
  ksg_node_view* nodes;
  ksg_pod_view* pods;
  int32_t* bound_node; /* pods [0, n_bound) run on these nodes */
} scenario;

static ksg_plugin_view* plugins(int n, const char** names, const int* w) {
  ksg_plugin_view* p = A(n, sizeof *p);
  for (int i = 0; i < n; i++) { p[i].name = names[i]; p[i].weight = w[i]; }
  return p;
}
static void default_args(ksg_profile_view* pv) {
  static ksg_quantity cm[2] = {{"cpu", 1}, {"memory", 1}};
  pv->fit_strategy = "LeastAllocated";
  pv->n_fit_resources = 2; pv->fit_resources = cm;
  pv->n_ba_resources = 2; pv->ba_resources = cm;
  pv->hard_pod_affinity_weight = 1;
  pv->pts_system_defaulted = 1;
}

static ksg_node_view make_node(int i, int zones, int tainted) {
  static const char* itype[] = {"m5.large", "m5.xlarge", "m6.2xlarge", "m6.4xlarge"};
  ksg_node_view n;
  memset(&n, 0, sizeof n);
  n.name = S("node-%04d", i);
  ksg_str_pair* l = A(4, sizeof *l);
  l[0] = (ksg_str_pair){"kubernetes.io/hostname", n.name};
  l[1] = (ksg_str_pair){"topology.kubernetes.io/zone", S("zone-%d", i % zones)};
  l[2] = (ksg_str_pair){"node.kubernetes.io/instance-type", itype[rnd(4)]};
  l[3] = (ksg_str_pair){"pool", S("pool-%d", rnd(6))};
  n.n_labels = 4; n.labels = l;
  ksg_quantity* q = A(4, sizeof *q);
  static const int64_t cores[] = {8, 16, 32, 64}, mem[] = {32, 64, 128, 256};
  q[0] = (ksg_quantity){"cpu", cores[rnd(4)] * 1000};
  q[1] = (ksg_quantity){"memory", mem[rnd(4)] * GI};
  q[2] = (ksg_quantity){"ephemeral-storage", 200 * GI};
  q[3] = (ksg_quantity){"pods", 110};
  n.n_alloc = 4; n.allocatable = q;
  if (tainted) {
    const uint32_t u = rnd(10);
    if (u == 0 || u == 1) {
      ksg_taint_view* t = A(1, sizeof *t);
      if (u == 0) *t = (ksg_taint_view){"dedicated", l[3].value, "NoSchedule"};
      else *t = (ksg_taint_view){"spot", "true", "PreferNoSchedule"};
      n.n_taints = 1; n.taints = t;
    }
  }
  if (rnd(3) == 0) {
    ksg_image_view* im = A(1, sizeof *im);
    const char** nm = A(1, sizeof *nm);
    nm[0] = "registry.example.com/app:v1";
    im->n_names = 1; im->names = nm; im->size_bytes = (100 + rnd(800)) * MI;
    n.n_images = 1; n.images = im;
  }
  return n;
}

static ksg_container_view* one_container(int best_effort) {
  static const int64_t cpu[] = {100, 250, 500, 1000, 2000}, mem[] = {128, 256, 512, 1024, 4096};
  ksg_container_view* c = A(1, sizeof *c);
  c->image = rnd(2) ? "registry.example.com/app:v1" : "registry.k8s.io/pause:3.10";
  if (!best_effort) {
    ksg_quantity* q = A(2, sizeof *q);
    q[0] = (ksg_quantity){"cpu", cpu[rnd(5)]};
    q[1] = (ksg_quantity){"memory", mem[rnd(5)] * MI};
    c->n_requests = 2; c->requests = q;
  }
  return c;
}

static ksg_requirement_view* req_in(const char* key, int nv, const char** vals) {
  ksg_requirement_view* r = A(1, sizeof *r);
  r->key = key; r->op = "In"; r->n_values = nv; r->values = vals;
  return r;
}

/* config-2 style: Fit + BalancedAllocation + TaintToleration + NodeAffinity */
static scenario scenario_c2(int N, int P, int bound) {
  scenario s;
  memset(&s, 0, sizeof s);
  s.name = "c2";
  static const char* names[] = {"PrioritySort", "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity",
                                "NodeResourcesFit", "NodeResourcesBalancedAllocation", "DefaultBinder"};
  static const int w[] = {0, 0, 0, 3, 2, 1, 1, 0};
  s.prof.n_plugins = 8; s.prof.plugins = plugins(8, names, w);
  default_args(&s.prof);
  s.n_nodes = N; s.n_pods = P; s.n_bound = bound;
  s.nodes = A(N, sizeof *s.nodes);
  for (int i = 0; i < N; i++) s.nodes[i] = make_node(i, 4, 1);
  s.pods = A(P, sizeof *s.pods);
  s.bound_node = A(bound, sizeof *s.bound_node);
  for (int j = 0; j < P; j++) {
    ksg_pod_view* p = &s.pods[j];
    p->namespace_ = "default";
    p->name = S("pod-%05d", j);
    p->n_containers = 1;
    p->containers = one_container(rnd(20) == 0);
    p->node_name = "";
    if (rnd(10) < 3) {
      ksg_toleration_view* t = A(2, sizeof *t);
      if (rnd(2)) {
        t[0] = (ksg_toleration_view){"dedicated", "Equal", S("pool-%d", rnd(6)), "NoSchedule"};
        p->n_tolerations = 1;
      } else {
        t[0] = (ksg_toleration_view){"spot", "Exists", "", ""};
        t[1] = (ksg_toleration_view){"dedicated", "Exists", "", "NoSchedule"};
        p->n_tolerations = 2;
      }
      p->tolerations = t;
    }
    if (rnd(4) == 0) {
      const char** z = A(2, sizeof *z);
      z[0] = S("zone-%d", rnd(4));
      z[1] = S("zone-%d", rnd(4));
      ksg_node_selector_term_view* term = A(1, sizeof *term);
      term->n_expr = 1; term->expr = req_in("topology.kubernetes.io/zone", 2, z);
      p->has_na_required = 1; p->n_na_required = 1; p->na_required = term;
    }
    if (rnd(4) == 0) {
      static const char* it[] = {"m5.large", "m6.4xlarge"};
      ksg_preferred_term_view* pt = A(1, sizeof *pt);
      pt->weight = 1 + rnd(100);
      pt->preference.n_expr = 1;
      pt->preference.expr = req_in("node.kubernetes.io/instance-type", 1, &it[rnd(2)]);
      p->has_na_preferred = 1; p->n_na_preferred = 1; p->na_preferred = pt;
    }
    if (rnd(10) == 0) {
      ksg_str_pair* ns = A(1, sizeof *ns);
      *ns = (ksg_str_pair){"pool", S("pool-%d", rnd(6))};
      p->has_node_selector = 1; p->n_node_selector = 1; p->node_selector = ns;
    }
    if (j < bound) {
      s.bound_node[j] = (int32_t)rnd(N);
      p->node_name = s.nodes[s.bound_node[j]].name;
    }
  }
  return s;
}

/* config-3 style: PodTopologySpread + InterPodAffinity over zone / hostname */
static scenario scenario_c3(int N, int P, int bound, int apps) {
  scenario s = scenario_c2(N, P, 0);
  s.name = "c3";
  static const char* names[] = {"PrioritySort", "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity",
                                "NodeResourcesFit", "PodTopologySpread", "InterPodAffinity",
                                "NodeResourcesBalancedAllocation", "DefaultBinder"};
  static const int w[] = {0, 0, 0, 3, 2, 1, 2, 2, 1, 0};
  s.prof.n_plugins = 10; s.prof.plugins = plugins(10, names, w);
  s.n_bound = bound;
  s.bound_node = A(bound, sizeof *s.bound_node);
  for (int j = 0; j < P; j++) {
    ksg_pod_view* p = &s.pods[j];
    const int a = (int)rnd(apps);
    ksg_str_pair* lab = A(1, sizeof *lab);
    *lab = (ksg_str_pair){"app", S("app-%02d", a)};
    p->n_labels = 1; p->labels = lab;
    ksg_label_selector_view sel;
    memset(&sel, 0, sizeof sel);
    sel.is_set = 1; sel.n_labels = 1; sel.match_labels = lab;
    ksg_spread_view* sp = A(2, sizeof *sp);
    sp[0] = (ksg_spread_view){5, "topology.kubernetes.io/zone", "ScheduleAnyway", sel, 0, NULL, NULL, 0, NULL};
    sp[1] = (ksg_spread_view){1 + (int)rnd(2), "kubernetes.io/hostname", "DoNotSchedule", sel, 0, NULL, NULL, 0, NULL};
    p->n_spread = 2; p->spread = sp;
    if (rnd(10) < 3) {
      ksg_affinity_term_view* t = A(1, sizeof *t);
      t->weight = 1 + rnd(100); t->selector = sel; t->topology_key = "kubernetes.io/hostname";
      p->n_pod_anti_affinity_preferred = 1; p->pod_anti_affinity_preferred = t;
    }
    if (rnd(10) == 0) {
      ksg_str_pair* o = A(1, sizeof *o);
      *o = (ksg_str_pair){"app", S("app-%02d", (a + 1 + (int)rnd(apps - 1)) % apps)};
      ksg_affinity_term_view* t = A(1, sizeof *t);
      t->selector.is_set = 1; t->selector.n_labels = 1; t->selector.match_labels = o;
      t->topology_key = "topology.kubernetes.io/zone";
      p->n_pod_affinity_required = 1; p->pod_affinity_required = t;
    }
    if (j < bound) {
      s.bound_node[j] = (int32_t)rnd(N);
      p->node_name = s.nodes[s.bound_node[j]].name;
    }
  }
  return s;
}

/* README.md:56-81 example: two 4-CPU / 32Gi nodes, a 100m / 16Gi pause pod,
 * the default profile (scheduler_test.go:519-541 order and weights). */
static scenario scenario_kat(void) {
  scenario s;
  memset(&s, 0, sizeof s);
  s.name = "kat";
  static const char* names[] = {"SchedulingGates", "PrioritySort", "NodeUnschedulable", "NodeName",
                                "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
                                "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding", "VolumeZone",
                                "PodTopologySpread", "InterPodAffinity", "DefaultPreemption",
                                "NodeResourcesBalancedAllocation", "ImageLocality", "DefaultBinder"};
  static const int w[] = {0, 0, 0, 0, 3, 2, 0, 1, 0, 0, 0, 0, 2, 2, 0, 1, 1, 0};
  s.prof.n_plugins = 18; s.prof.plugins = plugins(18, names, w);
  default_args(&s.prof);
  s.n_nodes = 2; s.n_pods = 1;
  s.nodes = A(2, sizeof *s.nodes);
  for (int i = 0; i < 2; i++) {
    ksg_node_view* n = &s.nodes[i];
    n->name = i ? "node-gp9t4" : "node-282x7";
    ksg_str_pair* l = A(1, sizeof *l);
    *l = (ksg_str_pair){"kubernetes.io/hostname", n->name};
    n->n_labels = 1; n->labels = l;
    ksg_quantity* q = A(3, sizeof *q);
    q[0] = (ksg_quantity){"cpu", 4000};
    q[1] = (ksg_quantity){"memory", 32 * GI};
    q[2] = (ksg_quantity){"pods", 110};
    n->n_alloc = 3; n->allocatable = q;
  }
  s.pods = A(1, sizeof *s.pods);
  ksg_container_view* c = A(1, sizeof *c);
  ksg_quantity* rq = A(2, sizeof *rq);
  rq[0] = (ksg_quantity){"cpu", 100};
  rq[1] = (ksg_quantity){"memory", 16 * GI};
  c->image = "registry.k8s.io/pause:3.5"; c->n_requests = 2; c->requests = rq;
  s.pods[0].namespace_ = "default"; s.pods[0].name = "hoge-pod"; s.pods[0].node_name = "";
  s.pods[0].n_containers = 1; s.pods[0].containers = c;
  return s;
}

/* ---- the reference's export sample profile (tests/golden/export_profile.txt,
 * written by tests/golden/make_export_profile.py from export.md:32): the view a
 * Go caller builds after ConvertForSimulator, per-point sets included ---- */
static const char* g_export_path = NULL;

static int load_export_profile(const char* path, ksg_profile_view* pv) {
  static const char* pts[KSG_NPOINTS] = {"preFilter", "filter", "preScore", "score"};
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  memset(pv, 0, sizeof *pv);
  ksg_plugin_view* mp = A(64, sizeof *mp);
  ksg_plugin_view* en[KSG_NPOINTS];
  const char** dis[KSG_NPOINTS];
  for (int k = 0; k < KSG_NPOINTS; k++) { en[k] = A(32, sizeof **en); dis[k] = A(32, sizeof **dis); }
  ksg_quantity* fr = A(8, sizeof *fr);
  ksg_quantity* br = A(8, sizeof *br);
  char line[512], a[128], b[128], c[128];
  while (fgets(line, sizeof line, f)) {
    if (line[0] == '#' || line[0] == '\n') continue;
    int w = 0, k;
    if (sscanf(line, "multipoint %127s %d", a, &w) == 2) {
      mp[pv->n_plugins++] = (ksg_plugin_view){strdup(a), w};
    } else if (sscanf(line, "enabled %127s %127s %d", a, b, &w) == 3) {
      for (k = 0; k < KSG_NPOINTS && strcmp(a, pts[k]); k++) {}
      if (k == KSG_NPOINTS) return -1;
      en[k][pv->points[k].n_enabled++] = (ksg_plugin_view){strdup(b), w};
      pv->points[k].enabled = en[k];
    } else if (sscanf(line, "disabled %127s %127s", a, b) == 2) {
      for (k = 0; k < KSG_NPOINTS && strcmp(a, pts[k]); k++) {}
      if (k == KSG_NPOINTS) return -1;
      dis[k][pv->points[k].n_disabled++] = strdup(b);
      pv->points[k].disabled = dis[k];
    } else if (sscanf(line, "fit_strategy %127s", a) == 1) {
      pv->fit_strategy = strdup(a);
    } else if (sscanf(line, "fit_resource %127s %d", a, &w) == 2) {
      fr[pv->n_fit_resources++] = (ksg_quantity){strdup(a), w};
      pv->fit_resources = fr;
    } else if (sscanf(line, "ba_resource %127s %d", a, &w) == 2) {
      br[pv->n_ba_resources++] = (ksg_quantity){strdup(a), w};
      pv->ba_resources = br;
    } else if (sscanf(line, "hard_pod_affinity_weight %d", &w) == 1) {
      pv->hard_pod_affinity_weight = w;
    } else if (sscanf(line, "ignore_preferred_terms_of_existing_pods %d", &w) == 1) {
      pv->ignore_preferred_terms_of_existing_pods = w;
    } else if (sscanf(line, "pts_system_defaulted %d", &w) == 1) {
      pv->pts_system_defaulted = w;
    } else if (sscanf(line, "%127s %127s %127s", a, b, c) >= 1) {
      fclose(f);
      return -1;
    }
  }
  fclose(f);
  pv->plugins = mp;
  return pv->n_plugins > 0 ? 0 : -1;
}

static ksg_snapshot* build(const scenario* s, int n_pods) {
  ksg_snapshot* snap;
  OK(ksg_snapshot_new(&s->prof, &snap));
  for (int i = 0; i < s->n_nodes; i++) OK(ksg_snapshot_add_node(snap, &s->nodes[i], NULL));
  for (int j = 0; j < n_pods; j++) OK(ksg_snapshot_add_pod(snap, &s->pods[j], NULL));
  for (int j = 0; j < s->n_bound; j++) OK(ksg_snapshot_bind(snap, j, s->bound_node[j]));
  return snap;
}

static kso_ctx* oracle_of(ksg_snapshot* snap, const scenario* s) {
  ksg_nodes nd;
  ksg_topology tp;
  ksg_workload wl;
  ksg_profile pf;
  OK(ksg_snapshot_view(snap, &nd, &tp, &wl, &pf));
  kso_ctx* o;
  OK(kso_open(4, &o));
  OK(kso_set_profile(o, &pf));
  OK(kso_load_nodes(o, &nd, &tp));
  OK(kso_load_workload(o, &wl));
  for (int j = 0; j < s->n_bound; j++) OK(kso_commit(o, j, s->bound_node[j]));
  return o;
}

/* README KAT (README.md:66,80): NodeResourcesFit raw 73, BalancedAllocation
 * raw 76, TaintToleration normalised 100 (final 300 at weight 3). */
static void check_kat(void) {
  scenario s = scenario_kat();
  ksg_snapshot* snap = build(&s, 1);
  OK(ksg_snapshot_encode(snap));
  kso_ctx* o = oracle_of(snap, &s);
  uint32_t fs[2];
  int64_t raw[KSG_NPLUGINS * 2], norm[KSG_NPLUGINS * 2], tot[2];
  ksg_capture cap = {fs, raw, norm, tot};
  ksg_result r;
  OK(kso_eval(o, 0, &r, &cap));
  CHECK(r.n_feasible == 2, "kat feasible %d", r.n_feasible);
  CHECK(raw[KSG_PL_NODE_RESOURCES_FIT * 2] == 73, "kat Fit %lld", (long long)raw[KSG_PL_NODE_RESOURCES_FIT * 2]);
  CHECK(raw[KSG_PL_BALANCED_ALLOCATION * 2] == 76, "kat BA %lld", (long long)raw[KSG_PL_BALANCED_ALLOCATION * 2]);
  CHECK(norm[KSG_PL_TAINT_TOLERATION * 2] == 100, "kat taint norm %lld", (long long)norm[KSG_PL_TAINT_TOLERATION * 2]);
  int32_t code, has, n;
  OK(ksg_snapshot_prefilter(snap, 0, KSG_PL_POD_TOPOLOGY_SPREAD, r.status, &code, &has, NULL, 0, &n));
  CHECK(code == KSG_CODE_SKIP, "kat PTS prefilter code %d", code);
  OK(ksg_snapshot_prefilter(snap, 0, KSG_PL_NODE_RESOURCES_FIT, r.status, &code, &has, NULL, 0, &n));
  CHECK(code == KSG_CODE_SUCCESS, "kat Fit prefilter code %d", code);
  printf("ok kat: Fit 73, BalancedAllocation 76, TaintToleration 100\n");
  kso_close(o);
  ksg_snapshot_free(snap);
}

/* The volume plugins through the C ABI alone (ksg_snapshot_add_pv / _pvc /
 * _storage_class): a local PV pinned to node-0001 (VolumeBinding's
 * PreFilterResult), a missing claim (VolumeRestrictions' PreFilter
 * rejection and its message), a zonal PV in z0 (VolumeZone at Filter), an
 * unbound WaitForFirstConsumer claim whose class allows z1 only
 * (VolumeBinding's BindConflict at Filter); decisions from the oracle on the
 * native encoding, messages from ksg_snapshot_status. */
static void check_volumes(void) {
  scenario s = scenario_kat();   /* the in-tree default plugin set, volume plugins included */
  s.n_nodes = 4;
  s.nodes = A(4, sizeof *s.nodes);
  for (int i = 0; i < 4; i++) {
    ksg_node_view* n = &s.nodes[i];
    n->name = S("node-%04d", i);
    ksg_str_pair* l = A(2, sizeof *l);
    l[0] = (ksg_str_pair){"kubernetes.io/hostname", n->name};
    l[1] = (ksg_str_pair){"topology.kubernetes.io/zone", i < 2 ? "z0" : "z1"};
    n->n_labels = 2; n->labels = l;
    ksg_quantity* q = A(3, sizeof *q);
    q[0] = (ksg_quantity){"cpu", 4000};
    q[1] = (ksg_quantity){"memory", 32 * GI};
    q[2] = (ksg_quantity){"pods", 110};
    n->n_alloc = 3; n->allocatable = q;
  }
  ksg_snapshot* snap = build(&s, 0);
  static ksg_str_pair done[1] = {{"pv.kubernetes.io/bind-completed", "yes"}};
  static const char* rwo[1] = {"ReadWriteOnce"};
  /* pv-local: required node affinity hostname In [node-0001] */
  static const char* host1[1] = {"node-0001"};
  ksg_node_selector_term_view term = {1, req_in("kubernetes.io/hostname", 1, host1), 0, NULL};
  ksg_pv_view pv_local = {"pv-local", 0, NULL, "", "default", "pvc-local", "local", 1, 1, &term};
  static ksg_str_pair zl[1] = {{"topology.kubernetes.io/zone", "z0"}};
  ksg_pv_view pv_zonal = {"pv-zonal", 1, zl, "", "default", "pvc-zonal", "csi", 0, 0, NULL};
  OK(ksg_snapshot_add_pv(snap, &pv_local));
  OK(ksg_snapshot_add_pv(snap, &pv_zonal));
  ksg_pvc_view c_local = {"default", "pvc-local", "pv-local", "", 1, rwo, 1, done, 0};
  ksg_pvc_view c_zonal = {"default", "pvc-zonal", "pv-zonal", "", 1, rwo, 1, done, 0};
  ksg_pvc_view c_wffc = {"default", "pvc-wffc", "", "wffc", 1, rwo, 0, NULL, 0};
  OK(ksg_snapshot_add_pvc(snap, &c_local));
  OK(ksg_snapshot_add_pvc(snap, &c_zonal));
  OK(ksg_snapshot_add_pvc(snap, &c_wffc));
  static const char* z1[1] = {"z1"};
  ksg_topology_requirement_view treq = {"topology.kubernetes.io/zone", 1, z1};
  ksg_topology_term_view tterm = {1, &treq};
  ksg_storage_class_view sc = {"wffc", "csi.example.com", "WaitForFirstConsumer", 1, &tterm};
  OK(ksg_snapshot_add_storage_class(snap, &sc));
  static const char* claims[4] = {"pvc-local", "missing", "pvc-zonal", "pvc-wffc"};
  ksg_pod_view pods[4];
  for (int j = 0; j < 4; j++) {
    pods[j] = s.pods[0];
    pods[j].name = S("claims-%d", j);
    ksg_volume_view* v = A(1, sizeof *v);
    v->name = "data"; v->kind = "persistentVolumeClaim"; v->claim_name = claims[j];
    pods[j].n_volumes = 1; pods[j].volumes = v;
    OK(ksg_snapshot_add_pod(snap, &pods[j], NULL));
  }
  OK(ksg_snapshot_encode(snap));
  s.n_pods = 0;
  kso_ctx* o = oracle_of(snap, &s);
  uint32_t fs[4][4];
  ksg_result r[4];
  for (int j = 0; j < 4; j++) {
    int64_t raw[KSG_NPLUGINS * 4], norm[KSG_NPLUGINS * 4], tot[4];
    ksg_capture cap = {fs[j], raw, norm, tot};
    OK(kso_eval(o, j, &r[j], &cap));
  }
  int32_t code, has, n;
  const char* names[4];
  OK(ksg_snapshot_prefilter(snap, 0, KSG_PL_VOLUME_BINDING, r[0].status, &code, &has, names, 4, &n));
  CHECK(code == KSG_CODE_SUCCESS && has == 1 && n == 1 && strcmp(names[0], "node-0001") == 0,
        "volumes: VolumeBinding PreFilterResult code %d has %d n %d", code, has, n);
  CHECK(r[0].n_feasible == 1 && r[0].selected == 1, "volumes: local PV pod feasible %d selected %d",
        r[0].n_feasible, r[0].selected);
  OK(ksg_snapshot_prefilter(snap, 1, KSG_PL_VOLUME_RESTRICTIONS, r[1].status, &code, &has, NULL, 0, &n));
  CHECK(code == KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE, "volumes: missing claim PreFilter code %d", code);
  char msg[256];
  int32_t len;
  OK(ksg_snapshot_prefilter_message(snap, 1, KSG_PL_VOLUME_RESTRICTIONS, msg, sizeof msg, &len));
  CHECK(strcmp(msg, "persistentvolumeclaim \"missing\" not found") == 0, "volumes: message '%s'", msg);
  CHECK(r[1].n_feasible == 0 && fs[1][0] == KSG_FS_NOT_EVALUATED, "volumes: rejected pod evaluated a node");
  /* pv-zonal in z0: nodes 2, 3 fail VolumeZone */
  CHECK(r[2].n_feasible == 2 && fs[2][0] == 0 && (fs[2][2] & 0xff) == KSG_PL_VOLUME_ZONE + 1,
        "volumes: zonal feasible %d word %#x", r[2].n_feasible, fs[2][2]);
  OK(ksg_snapshot_status(snap, 2, fs[2][2], 2, &code, msg, sizeof msg, &len));
  CHECK(code == KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE && strcmp(msg, "node(s) had no available volume zone") == 0,
        "volumes: zone status %d '%s'", code, msg);
  /* the class allows z1: nodes 0, 1 cannot provision */
  CHECK(r[3].n_feasible == 2 && fs[3][3] == 0 && (fs[3][0] & 0xff) == KSG_PL_VOLUME_BINDING + 1,
        "volumes: WaitForFirstConsumer feasible %d word %#x", r[3].n_feasible, fs[3][0]);
  OK(ksg_snapshot_status(snap, 3, fs[3][0], 0, &code, msg, sizeof msg, &len));
  CHECK(strcmp(msg, "node(s) didn't find available persistent volumes to bind") == 0, "volumes: bind status '%s'",
        msg);
  printf("ok volumes: VolumeBinding result {node-0001}, VolumeRestrictions rejection, VolumeZone and "
         "BindConflict at Filter\n");
  kso_close(o);
  ksg_snapshot_free(snap);
}

/* Incremental encoding (pods added after the first encode) against one full
 * encode: identical pod records and program pool when appended. */
static void check_incremental_bytes(const scenario* s) {
  ksg_snapshot* full = build(s, s->n_pods);
  OK(ksg_snapshot_encode(full));
  ksg_snapshot* inc = build(s, s->n_bound + 1);
  OK(ksg_snapshot_encode(inc));
  int appended = 0, reloads = 0;
  for (int j = s->n_bound + 1; j < s->n_pods; j++) {
    int32_t ap;
    OK(ksg_snapshot_add_pod(inc, &s->pods[j], NULL));
    OK(ksg_snapshot_encode_incremental(inc, &ap));
    appended += ap;
    reloads += !ap;
  }
  ksg_workload a, b;
  OK(ksg_snapshot_view(full, NULL, NULL, &a, NULL));
  OK(ksg_snapshot_view(inc, NULL, NULL, &b, NULL));
  CHECK(a.n_pods == b.n_pods && a.prog_len == b.prog_len, "%s: sizes differ", s->name);
  CHECK(a.n_pods == b.n_pods && memcmp(a.pods, b.pods, sizeof(ksg_pod) * a.n_pods) == 0, "%s: pod records differ",
        s->name);
  CHECK(a.prog_len == b.prog_len && memcmp(a.prog, b.prog, 4 * a.prog_len) == 0, "%s: programs differ", s->name);
  printf("ok %s incremental encoding: %d appended, %d full re-encodes, bytes identical\n", s->name, appended, reloads);
  ksg_snapshot_free(full);
  ksg_snapshot_free(inc);
}

static void oracle_queue(kso_ctx* o, const scenario* s, int32_t* pl, ksg_result* res) {
  OK(kso_run_queue(o, s->n_bound, s->n_pods - s->n_bound, pl, res, NULL));
}

static int run_cpu(void) {
  check_kat();
  check_volumes();
  scenario sc[2] = {scenario_c2(96, 400, 24), scenario_c3(64, 300, 16, 8)};
  for (int k = 0; k < 2; k++) {
    const scenario* s = &sc[k];
    check_incremental_bytes(s);
    ksg_snapshot* snap = build(s, s->n_pods);
    OK(ksg_snapshot_encode(snap));
    kso_ctx* o = oracle_of(snap, s);
    const int Q = s->n_pods - s->n_bound;
    int32_t* pl = A(Q, 4);
    ksg_result* res = A(Q, sizeof *res);
    oracle_queue(o, s, pl, res);
    int placed = 0;
    for (int i = 0; i < Q; i++) placed += pl[i] >= 0;
    CHECK(placed > Q / 2, "%s: only %d of %d placed", s->name, placed, Q);
    printf("ok %s oracle queue: %d of %d pods placed\n", s->name, placed, Q);
    kso_close(o);
    ksg_snapshot_free(snap);
  }
  return g_fail;
}

static int run_gpu(void) {
  scenario sc[2] = {scenario_c2(96, 400, 24), scenario_c3(64, 300, 16, 8)};
  for (int k = 0; k < 2; k++) {
    const scenario* s = &sc[k];
    const int N = s->n_nodes, Q = s->n_pods - s->n_bound;
    /* (1) whole queue on the device vs the oracle */
    ksg_snapshot* snap = build(s, s->n_pods);
    ksg_ctx* ctx;
    OK(ksg_open(0, &ctx));
    if (ksg_snapshot_load(snap, ctx)) {
      fprintf(stderr, "load: %s\n", ksg_snapshot_error(snap));
      return 2;
    }
    int32_t* pl = A(Q, 4);
    int32_t* want = A(Q, 4);
    ksg_result* res = A(Q, sizeof *res);
    ksg_result* wres = A(Q, sizeof *wres);
    OK(ksg_run_queue(ctx, s->n_bound, Q, pl, res, NULL));
    kso_ctx* o = oracle_of(snap, s);
    oracle_queue(o, s, want, wres);
    int bad = 0;
    for (int i = 0; i < Q; i++)
      bad += pl[i] != want[i] || res[i].n_feasible != wres[i].n_feasible || res[i].status != wres[i].status ||
             res[i].score_skip != wres[i].score_skip;
    CHECK(bad == 0, "%s: %d of %d pods differ from the oracle (ksg_run_queue)", s->name, bad, Q);
    printf("ok %s ksg_run_queue: %d pods identical to the oracle\n", s->name, Q);
    kso_close(o);
    ksg_close(ctx);

    /* (2) the per-cycle path of the Go shim: add_pod -> sync -> ksg_eval ->
     * status words / messages -> assume, one pod at a time */
    ksg_snapshot* cyc = build(s, s->n_bound);
    OK(ksg_open(0, &ctx));
    if (ksg_snapshot_load(cyc, ctx)) {
      fprintf(stderr, "load: %s\n", ksg_snapshot_error(cyc));
      return 2;
    }
    o = oracle_of(snap, s);
    uint32_t* fs = A(N, 4);
    uint32_t* wfs = A(N, 4);
    ksg_capture cap = {fs, NULL, NULL, NULL}, wcap = {wfs, NULL, NULL, NULL};
    int appended = 0, mismatch = 0, msgs = 0;
    char msg[512];
    for (int j = s->n_bound; j < s->n_pods; j++) {
      int32_t idx, ap;
      OK(ksg_snapshot_add_pod(cyc, &s->pods[j], &idx));
      if (ksg_snapshot_sync(cyc, ctx, &ap)) {
        fprintf(stderr, "sync: %s\n", ksg_snapshot_error(cyc));
        return 2;
      }
      appended += ap;
      ksg_result r, wr;
      OK(ksg_eval(ctx, idx, &r, &cap));
      OK(kso_eval(o, j, &wr, &wcap));
      if (r.selected != wr.selected || r.n_feasible != wr.n_feasible || memcmp(fs, wfs, 4 * N) != 0) mismatch++;
      for (int n = 0; n < N; n++) {
        if (fs[n] == 0 || fs[n] == KSG_FS_NOT_EVALUATED) continue;
        int32_t code, len;
        OK(ksg_snapshot_status(cyc, idx, fs[n], n, &code, msg, sizeof msg, &len));
        CHECK(len > 0 && (code == KSG_CODE_UNSCHEDULABLE || code == KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE),
              "%s: status of pod %d node %d: code %d '%s'", s->name, j, n, code, msg);
        msgs++;
      }
      if (r.selected >= 0) {
        OK(ksg_snapshot_assume(cyc, ctx, idx, r.selected));
        OK(kso_commit(o, j, r.selected));
      }
    }
    CHECK(mismatch == 0, "%s: %d of %d cycles differ from the oracle (per-cycle path)", s->name, mismatch, Q);
    printf("ok %s per-cycle path: %d cycles (%d appended, %d reloads), status words identical, %d messages\n",
           s->name, Q, appended, Q - appended, msgs);
    kso_close(o);
    ksg_close(ctx);
    ksg_snapshot_free(cyc);
    ksg_snapshot_free(snap);
  }
  return g_fail;
}

/* ---- annotations of one cycle through ksg_annotate, with the profile's
 * derived orders and the Store's weight map (ksg_snapshot_profile_info) ---- */
typedef struct {
  const char* s[3];
  int64_t len[3];
} ann3;

static ksg_annotator* annotator_of(ksg_snapshot* snap) {
  static const char* plugin_names[KSG_NPLUGINS] = {
      "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
      "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread",
      "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"};
  int32_t N, P, R, T;
  OK(ksg_snapshot_counts(snap, &N, &P, &R, &T));
  const char** node = A(N, sizeof *node);
  const char** res = A(R, sizeof *res);
  const char** taint = A(T ? T : 1, sizeof *taint);
  OK(ksg_snapshot_names(snap, node, res, taint));
  ksg_nodes nd;
  OK(ksg_snapshot_view(snap, &nd, NULL, NULL, NULL));
  ksg_names nm = {N, node, plugin_names, R, res, T, taint, nd.max_taints, nd.taints};
  ksg_annotator* an;
  OK(ksg_annotator_new(&nm, &an));
  return an;
}

/* filter-result / score-result / finalscore-result of one cycle; the strings
 * are copied (the annotator owns its buffers until the next call) */
static ann3 annotate(ksg_annotator* an, const ksg_profile_info* info, const ksg_pod* pod, const ksg_result* r,
                     const ksg_capture* cap) {
  int32_t fo[KSG_NPLUGINS], so[KSG_NPLUGINS], nf = 0, ns = 0;
  uint32_t fskip = pod->filter_skip;
  if (r->status & KSG_ST_IPA_PREFILTER_SKIP) fskip |= 1u << KSG_PL_INTER_POD_AFFINITY;
  for (int k = 0; k < info->n_order[KSG_POINT_FILTER]; k++) {
    const int pl = info->order[KSG_POINT_FILTER][k];
    if (!((fskip >> pl) & 1u)) fo[nf++] = pl;
  }
  if (r->n_feasible >= 2)
    for (int k = 0; k < info->n_order[KSG_POINT_SCORE]; k++) {
      const int pl = info->order[KSG_POINT_SCORE][k];
      if (!((r->score_skip >> pl) & 1u)) so[ns++] = pl;
    }
  ksg_annotate_in in = {nf, fo, ns, so, info->normalize_mask, info->store_weight, r->n_feasible,
                        cap->fstatus, cap->raw, cap->norm};
  const char* js[3];
  int64_t ln[3];
  OK(ksg_annotate(an, &in, js, ln));
  ann3 out;
  for (int i = 0; i < 3; i++) {
    char* c = malloc(ln[i] + 1);
    memcpy(c, js[i], ln[i]);
    c[ln[i]] = 0;
    out.s[i] = c;
    out.len[i] = ln[i];
  }
  return out;
}

static void free_ann(ann3* a) {
  for (int i = 0; i < 3; i++) free((void*)a->s[i]);
}

/* Orders and weights the sample's profile must derive (the Python model pins
 * the same lists: tests/test_ingest.py test_export_sample_per_point_expansion). */
static void check_export_info(ksg_snapshot* snap, ksg_profile_info* info) {
  OK(ksg_snapshot_profile_info(snap, info));
  static const int filter[] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  static const int prefilter[] = {5, 4, 6, 10, 11, 8, 3, 7, 9};
  static const int prescore[] = {11, 10, 2, 3, 5, 8, 12};
  static const int score[] = {12, 13, 11, 5, 3, 10, 2, 8};
  const int* want[KSG_NPOINTS] = {prefilter, filter, prescore, score};
  const int nwant[KSG_NPOINTS] = {9, 12, 7, 8};
  for (int pt = 0; pt < KSG_NPOINTS; pt++) {
    int same = info->n_order[pt] == nwant[pt];
    for (int k = 0; same && k < nwant[pt]; k++) same = info->order[pt][k] == want[pt][k];
    CHECK(same, "export profile: point %d order differs", pt);
  }
  /* the Store keeps MultiPoint's weight, the framework the Score point's */
  CHECK(info->store_weight[KSG_PL_TAINT_TOLERATION] == 3 && info->selection_weight[KSG_PL_TAINT_TOLERATION] == 1,
        "export profile: TaintToleration weights %lld / %d", (long long)info->store_weight[KSG_PL_TAINT_TOLERATION],
        info->selection_weight[KSG_PL_TAINT_TOLERATION]);
  CHECK(info->store_weight[KSG_PL_POD_TOPOLOGY_SPREAD] == 2 && info->selection_weight[KSG_PL_POD_TOPOLOGY_SPREAD] == 2,
        "export profile: PodTopologySpread weights");
  CHECK(info->store_weight[KSG_PL_NODE_AFFINITY] == 2 && info->selection_weight[KSG_PL_NODE_AFFINITY] == 1,
        "export profile: NodeAffinity weights");
}

/* The sample's profile over a config-2 cluster (node-local pods: the
 * per-cycle chip-wide path) and a config-3 cluster (topology pods). */
static scenario scenario_export(int k, const ksg_profile_view* pv) {
  scenario s = k == 0 ? scenario_c2(96, 300, 24) : scenario_c3(64, 240, 16, 8);
  s.name = k == 0 ? "export-c2" : "export-c3";
  s.prof = *pv;
  return s;
}

static int run_export(int gpu) {
  ksg_profile_view pv;
  if (!g_export_path || load_export_profile(g_export_path, &pv)) {
    fprintf(stderr, "cannot read the export profile fixture %s\n", g_export_path ? g_export_path : "(none)");
    return 2;
  }
  for (int k = 0; k < 2; k++) {
    const scenario sc = scenario_export(k, &pv);
    const scenario* s = &sc;
    const int N = s->n_nodes, Q = s->n_pods - s->n_bound;
    ksg_snapshot* full = build(s, s->n_pods);
    ksg_profile_info info;
    check_export_info(full, &info);
    OK(ksg_snapshot_encode(full));
    kso_ctx* o = oracle_of(full, s);
    int32_t* want = A(Q, 4);
    ksg_result* wres = A(Q, sizeof *wres);
    oracle_queue(o, s, want, wres);
    kso_close(o);
    if (!gpu) {
      int placed = 0;
      for (int i = 0; i < Q; i++) placed += want[i] >= 0;
      CHECK(placed > 0, "%s: nothing placed", s->name);
      printf("ok %s profile info (per-point orders, store vs selection weights), oracle queue %d of %d placed\n",
             s->name, placed, Q);
      ksg_snapshot_free(full);
      continue;
    }
    /* (1) whole queue on the device */
    ksg_ctx* ctx;
    OK(ksg_open(0, &ctx));
    if (ksg_snapshot_load(full, ctx)) {
      fprintf(stderr, "load: %s\n", ksg_snapshot_error(full));
      return 2;
    }
    int32_t* pl = A(Q, 4);
    ksg_result* res = A(Q, sizeof *res);
    OK(ksg_run_queue(ctx, s->n_bound, Q, pl, res, NULL));
    int bad = 0;
    for (int i = 0; i < Q; i++)
      bad += pl[i] != want[i] || res[i].n_feasible != wres[i].n_feasible || res[i].status != wres[i].status ||
             res[i].score_skip != wres[i].score_skip;
    CHECK(bad == 0, "%s: %d of %d pods differ from the oracle (ksg_run_queue)", s->name, bad, Q);
    ksg_close(ctx);
    /* (2) the per-cycle path with capture, statuses and annotation bytes */
    ksg_snapshot* cyc = build(s, s->n_bound);
    OK(ksg_open(0, &ctx));
    if (ksg_snapshot_load(cyc, ctx)) {
      fprintf(stderr, "load: %s\n", ksg_snapshot_error(cyc));
      return 2;
    }
    o = oracle_of(full, s);
    uint32_t *fs = A(N, 4), *wfs = A(N, 4);
    int64_t *raw = A((size_t)KSG_NPLUGINS * N, 8), *norm = A((size_t)KSG_NPLUGINS * N, 8), *tot = A(N, 8);
    int64_t *wraw = A((size_t)KSG_NPLUGINS * N, 8), *wnorm = A((size_t)KSG_NPLUGINS * N, 8), *wtot = A(N, 8);
    ksg_capture cap = {fs, raw, norm, tot}, wcap = {wfs, wraw, wnorm, wtot};
    int32_t* codes = A(N, 4);
    int32_t* msgi = A(N, 4);
    char* msgs = A(1 << 16, 1);
    ksg_annotator* an = annotator_of(full);
    int mismatch = 0, ann_bad = 0, scored = 0, fast = 0;
    int64_t ann_bytes = 0;
    for (int j = s->n_bound; j < s->n_pods; j++) {
      int32_t idx, ap, path, flags, nm;
      int64_t ml;
      OK(ksg_snapshot_add_pod(cyc, &s->pods[j], &idx));
      if (ksg_snapshot_sync(cyc, ctx, &ap)) {
        fprintf(stderr, "sync: %s\n", ksg_snapshot_error(cyc));
        return 2;
      }
      memset(raw, 0, 8 * (size_t)KSG_NPLUGINS * N);
      memset(norm, 0, 8 * (size_t)KSG_NPLUGINS * N);
      memset(wraw, 0, 8 * (size_t)KSG_NPLUGINS * N);
      memset(wnorm, 0, 8 * (size_t)KSG_NPLUGINS * N);
      ksg_result r, wr;
      OK(ksg_eval(ctx, idx, &r, &cap));
      OK(ksg_last_run_info(ctx, &path, &flags));
      fast += path == 5;
      OK(kso_eval(o, j, &wr, &wcap));
      if (r.selected != wr.selected || r.n_feasible != wr.n_feasible || r.status != wr.status ||
          memcmp(fs, wfs, 4 * N) != 0)
        mismatch++;
      OK(ksg_snapshot_statuses(cyc, idx, fs, N, codes, msgi, msgs, 1 << 16, &nm, &ml));
      ksg_workload wl;
      OK(ksg_snapshot_view(cyc, NULL, NULL, &wl, NULL));
      ann3 a = annotate(an, &info, &wl.pods[idx], &r, &cap);
      ann3 b = annotate(an, &info, &wl.pods[idx], &wr, &wcap);
      for (int i = 0; i < 3; i++) {
        ann_bad += a.len[i] != b.len[i] || memcmp(a.s[i], b.s[i], a.len[i]) != 0;
        ann_bytes += a.len[i];
      }
      free_ann(&a);
      free_ann(&b);
      scored += r.n_feasible >= 2;
      if (r.selected >= 0) {
        OK(ksg_snapshot_assume(cyc, ctx, idx, r.selected));
        OK(kso_commit(o, j, r.selected));
      }
    }
    CHECK(mismatch == 0, "%s: %d of %d cycles differ from the oracle", s->name, mismatch, Q);
    CHECK(ann_bad == 0, "%s: %d annotation values differ from the oracle's", s->name, ann_bad);
    CHECK(k != 0 || fast == Q, "%s: %d of %d cycles on the per-cycle chip-wide path", s->name, fast, Q);
    printf("ok %s: ksg_run_queue identical; per-cycle path %d cycles (%d chip-wide, %d scored), status words and "
           "%lld annotation bytes identical to the oracle\n", s->name, Q, fast, scored, (long long)ann_bytes);
    ksg_annotator_free(an);
    kso_close(o);
    ksg_close(ctx);
    ksg_snapshot_free(cyc);
    ksg_snapshot_free(full);
  }
  return g_fail;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "--gpu") == 0;
  if (argc > 2) g_export_path = argv[2];
  int rc = gpu ? run_gpu() : run_cpu();
  if (rc == 0 && g_export_path) rc = run_export(gpu);
  printf(rc ? "FAILED (%d checks)\n" : "PASSED\n", rc);
  return rc ? 1 : 0;
}
