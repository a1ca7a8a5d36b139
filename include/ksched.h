/*
 * ksched.h — C ABI of the MI355X Filter/Score evaluator (libksched.so).
 *
 * Drop-in boundary for the debuggable scheduler's per-(pod, node, plugin) hot
 * path.  Today the upstream framework calls, per pod and per node, the wrapped
 * in-tree plugins:
 *   PreFilter       simulator/scheduler/plugin/wrappedplugin.go:491 (-> :504)
 *   Filter          simulator/scheduler/plugin/wrappedplugin.go:523 (-> :535)
 *   PreScore        simulator/scheduler/plugin/wrappedplugin.go:459 (-> :472)
 *   Score           simulator/scheduler/plugin/wrappedplugin.go:420 (-> :433)
 *   NormalizeScore  simulator/scheduler/plugin/wrappedplugin.go:388 (-> :400)
 *   Reserve/assume  simulator/scheduler/plugin/wrappedplugin.go:622 (AddSelectedNode)
 * and each call lands in Store (resultstore/store.go:423,461,481,522,537,562).
 * A cgo shim calls ksg_eval_view() ONCE per pod at PreFilter
 * time, stashes the returned SoA in CycleState, and answers every Filter /
 * Score / NormalizeScore call from it.  The shim has no Reserve plugin (it
 * would add an annotation entry upstream never writes): the assumed pod
 * reaches the device at the next cycle's snapshot diff, through
 * ksg_snapshot_assume -> ksg_commit().  ksg_run_queue()
 * runs a whole pod queue on the device (filter -> score -> normalise ->
 * weighted sum -> selectHost -> assume) without returning to the host.
 *
 * Conventions: all inputs are caller-owned and copied during the call; all
 * outputs go to caller-allocated buffers; no pointer is retained after return
 * (cgo pointer rules).  Every function returns 0 on success or a negative
 * KSG_E_* code; ksg_last_error() gives the message.  A context is not
 * thread-safe: the shim serialises calls (one call per pod).  No C++ exception
 * crosses this boundary.
 */
#ifndef KSCHED_H
#define KSCHED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSG_ABI_VERSION 4

#define KSG_OK 0
#define KSG_E_INVALID (-1)     /* bad argument / inconsistent sizes            */
#define KSG_E_DEVICE (-2)      /* HIP runtime error                            */
#define KSG_E_NOMEM (-3)       /* device or host allocation failed             */
#define KSG_E_STATE (-4)       /* call out of order (e.g. eval before load)    */
#define KSG_E_UNSUPPORTED (-5) /* input outside what the kernels implement     */
#define KSG_E_SCORE (-6)       /* a normalised score left [0,100] (framework error) */

/* Plugin ids (stable; profile.py uses the same numbering). */
enum {
  KSG_PL_NODE_UNSCHEDULABLE = 0,
  KSG_PL_NODE_NAME = 1,
  KSG_PL_TAINT_TOLERATION = 2,
  KSG_PL_NODE_AFFINITY = 3,
  KSG_PL_NODE_PORTS = 4,
  KSG_PL_NODE_RESOURCES_FIT = 5,
  KSG_PL_VOLUME_RESTRICTIONS = 6,
  KSG_PL_NODE_VOLUME_LIMITS = 7,
  KSG_PL_VOLUME_BINDING = 8,
  KSG_PL_VOLUME_ZONE = 9,
  KSG_PL_POD_TOPOLOGY_SPREAD = 10,
  KSG_PL_INTER_POD_AFFINITY = 11,
  KSG_PL_BALANCED_ALLOCATION = 12,
  KSG_PL_IMAGE_LOCALITY = 13,
  KSG_NPLUGINS = 14
};

#define KSG_MAX_RES 8      /* resource columns: 0 cpu (milli), 1 memory, 2 ephemeral, 3.. scalars */
#define KSG_RES_CPU 0
#define KSG_RES_MEM 1
#define KSG_RES_EPH 2

/* Taint effects (taint vocabulary). */
#define KSG_EFFECT_NO_SCHEDULE 1
#define KSG_EFFECT_PREFER_NO_SCHEDULE 2
#define KSG_EFFECT_NO_EXECUTE 3

/* ---- per-node filter status word --------------------------------------
 * (NodePorts: no payload; "node(s) didn't have free ports for the requested
 * pod ports", Unschedulable)
 * bits 0..7  : 0 = passed every filter that ran; else failing plugin id + 1
 * bits 8..31 : reason payload
 *   NodeResourcesFit : bit0 "Too many pods", bit1 cpu, bit2 memory, bit3
 *                      ephemeral-storage, bit(4+j) scalar column 3+j
 *   TaintToleration  : taint slot index on the node (message names the taint)
 *   NodeAffinity     : 1 = pod's affinity/selector
 *   PodTopologySpread: 1 = missing required label, 2 = skew
 *   InterPodAffinity : 1 affinity, 2 anti-affinity, 3 existing pods' anti-affinity
 * KSG_FS_NOT_EVALUATED: node outside the PreFilterResult node set (absent
 * from filter-result) or pod rejected at PreFilter.                         */
#define KSG_FS_NOT_EVALUATED 0xFFu

/* ---- cluster snapshot (SoA; column c of node i at [c * n_nodes + i]) ---- */
typedef struct ksg_nodes {
  int32_t n_nodes;
  int32_t n_res;                 /* <= KSG_MAX_RES                                 */
  const int64_t* alloc;          /* [n_res][n_nodes] allocatable                   */
  const int64_t* requested;      /* [n_res][n_nodes] NodeInfo.Requested            */
  const int64_t* nonzero;        /* [2][n_nodes]   NodeInfo.NonZeroRequested cpu,mem */
  const int32_t* allowed_pods;   /* [n_nodes]                                      */
  const int32_t* pod_count;      /* [n_nodes] len(NodeInfo.Pods)                   */
  const uint8_t* unschedulable;  /* [n_nodes] spec.unschedulable                   */
  int32_t n_label_cols;          /* label keys referenced by any selector / topology */
  const uint32_t* label_val;     /* [n_label_cols][n_nodes] value id, 0 = absent   */
  const int64_t* label_num;      /* [n_label_cols][n_nodes] strconv.ParseInt value */
  const uint8_t* label_num_ok;   /* [n_label_cols][n_nodes] parse succeeded        */
  int32_t max_taints;
  const uint32_t* taints;        /* [max_taints][n_nodes] taint-vocab id + 1 in node order, 0 = end */
  int32_t n_taint_vocab;
  const uint8_t* taint_effect;   /* [n_taint_vocab] KSG_EFFECT_*                   */
  int32_t max_images;
  const uint32_t* images;        /* [max_images][n_nodes] strictly ascending image id + 1, 0 = end */
  int32_t n_images;              /* image vocabulary size                          */
  int32_t n_port_vocab;          /* host-port vocabulary size (NodePorts): every (hostIP,
                                    protocol, hostPort) a pod uses; each node's UsedPorts is
                                    a bitmap over it, empty at load (bound pods are assumed) */
} ksg_nodes;

/* ---- topology tables for PodTopologySpread / InterPodAffinity ----------- */
#define KSG_TMPL_REQ_ANTI 0      /* existing pods' required anti-affinity term     */
#define KSG_TMPL_REQ_AFF 1       /* existing pods' required affinity term          */
#define KSG_TMPL_PREF 2          /* existing pods' preferred (anti-)affinity term  */
typedef struct ksg_topology {
  int32_t n_selectors;           /* pod label-selector ids (namespace-scoped)      */
  int32_t n_templates;           /* term templates owned by pods                   */
  const int32_t* tmpl_col;       /* [n_templates] label column of the topology key */
  const int32_t* tmpl_kind;      /* [n_templates] KSG_TMPL_*                       */
  const int32_t* tmpl_weight;    /* [n_templates] signed weight (PREF) or 1        */
  const int32_t* col_vocab;      /* [n_label_cols] value ids are < col_vocab[c]     */
  const uint8_t* col_unique;     /* [n_label_cols] every value on at most one node */
  const double* log_table;       /* [log_n] Go math.Log(float64(i)), i < log_n     */
  int32_t log_n;
} ksg_topology;

/* ---- pods ----------------------------------------------------------------
 * Encoded pod (152 B).  Variable-length parts live in a shared int32 program
 * pool; offsets are word indices into it, -1 = absent.  See encoder.py for
 * the program grammar.                                                      */
#define KSG_POD_TOL_UNSCHED (1u << 0)   /* tolerates node.kubernetes.io/unschedulable:NoSchedule */
#define KSG_POD_NA_REQUIRED (1u << 1)   /* has nodeSelector or required node affinity */
#define KSG_POD_BEST_EFFORT (1u << 2)   /* all BalancedAllocation resource requests zero */
#define KSG_POD_PREFILTER_REJECT (1u << 3) /* rejected at PreFilter: nothing evaluated */
typedef struct ksg_pod {
  int64_t req[KSG_MAX_RES];  /* PodRequests per resource column               */
  int64_t nz_cpu;            /* non-zero request (100m default per container)   */
  int64_t nz_mem;            /* non-zero request (200Mi default per container)  */
  uint32_t flags;            /* KSG_POD_*                                      */
  uint32_t filter_skip;      /* bit p: plugin p's PreFilter returned Skip      */
  uint32_t score_skip;       /* bit p: plugin p's PreScore returns Skip (host-decidable part) */
  int32_t node_name;         /* spec.nodeName as node index; -1 unset; -2 no such node */
  int32_t n_containers;      /* init + regular containers (ImageLocality)       */
  int32_t tol;               /* toleration bitmaps: [filter words][prefer words] */
  int32_t na_req;            /* required node affinity program                 */
  int32_t na_pref;           /* preferred node affinity program                */
  int32_t img;               /* ImageLocality program                          */
  int32_t node_set;          /* PreFilterResult node bitmap (n_nodes bits)      */
  int32_t pts;               /* PodTopologySpread program                      */
  int32_t ipa;               /* InterPodAffinity program                       */
  int32_t commit;            /* selectors matched + templates owned (assume)   */
  int32_t blob;              /* tol..ports programs are contiguous:            */
  int32_t blob_len;          /*   prog[blob, blob + blob_len) (staged into LDS) */
  int32_t ports;             /* NodePorts program: conflicting host-port ids, own ids */
  int32_t vol;               /* volume plugins' Filter program (pods with claims) */
  int32_t pad;
} ksg_pod;

typedef struct ksg_workload {
  const ksg_pod* pods;
  int32_t n_pods;
  const int32_t* prog;
  int64_t prog_len;
} ksg_workload;

/* ---- profile ------------------------------------------------------------ */
#define KSG_LEAST_ALLOCATED 0
#define KSG_MOST_ALLOCATED 1
#define KSG_REQUESTED_TO_CAPACITY_RATIO 2
#define KSG_MAX_SHAPE 16                 /* RequestedToCapacityRatio shape points  */
#define KSG_PROF_BA_SKIP_BEST_EFFORT (1u << 0)
#define KSG_PROF_IPA_IGNORE_EXISTING_PREF (1u << 1)
typedef struct ksg_profile {
  int32_t n_filter;
  int32_t filter_order[KSG_NPLUGINS];  /* Filter plugins in MultiPoint order      */
  uint32_t score_mask;                 /* bit p: plugin p runs at Score           */
  int32_t weight[KSG_NPLUGINS];        /* getScorePluginWeight (0 -> 1)           */
  int32_t fit_strategy;                /* KSG_LEAST_ALLOCATED / _MOST_ALLOCATED / _REQUESTED_TO_CAPACITY_RATIO */
  int32_t fit_n;
  int32_t fit_res[KSG_MAX_RES];        /* resource columns scored by Fit          */
  int64_t fit_w[KSG_MAX_RES];
  int32_t ba_n;
  int32_t ba_res[KSG_MAX_RES];         /* resource columns of BalancedAllocation  */
  int32_t hard_pod_affinity_weight;
  uint32_t flags;                      /* KSG_PROF_*                              */
  uint32_t fit_ignored_res;            /* bit r: scalar column r ignored by the Fit filter */
  int32_t shape_n;                     /* RequestedToCapacityRatio: shape points,   */
  int32_t shape_util[KSG_MAX_SHAPE];   /*   utilization 0..100 increasing, and the  */
  int32_t shape_score[KSG_MAX_SHAPE];  /*   score scaled to 0..100 (written x 10)   */
  int32_t pad;
} ksg_profile;

/* ---- per-pod results ------------------------------------------------------ */
#define KSG_ST_SCORED (1u << 0)          /* >= 2 feasible nodes: PreScore/Score ran */
#define KSG_ST_IPA_PREFILTER_SKIP (1u << 1)
#define KSG_ST_IPA_PRESCORE_SKIP (1u << 2)
#define KSG_ST_SCORE_ERROR (1u << 3)     /* normalised score outside [0,100]       */
typedef struct ksg_result {
  int32_t selected;     /* node index; -1 = unschedulable                      */
  int32_t n_feasible;
  uint32_t status;      /* KSG_ST_*                                             */
  uint32_t score_skip;  /* final PreScore Skip mask (host part | device part)   */
} ksg_result;

/* Optional capture of everything the wrapped plugins would record.  Arrays are
 * per pod; ksg_run_queue() writes pod k at offset k * (stride of the array).
 * raw / norm rows of plugins outside the profile's score set may be left
 * untouched (the batched path writes only the score set's rows). */
typedef struct ksg_capture {
  uint32_t* fstatus;    /* [n_nodes]                 filter status word       */
  int64_t* raw;         /* [KSG_NPLUGINS][n_nodes]   Score() value            */
  int64_t* norm;        /* [KSG_NPLUGINS][n_nodes]   after NormalizeScore     */
  int64_t* total;       /* [n_nodes]                 Σ normalised × weight    */
} ksg_capture;

/* Mutable node state, for read-back and checkpoints. */
typedef struct ksg_node_state {
  int64_t* requested;   /* [n_res][n_nodes] */
  int64_t* nonzero;     /* [2][n_nodes]     */
  int32_t* pod_count;   /* [n_nodes]        */
} ksg_node_state;

typedef struct ksg_replica_summary {
  int32_t scheduled;
  int32_t unschedulable;
  uint64_t placement_hash;   /* FNV-1a over the replica's placements  */
  int64_t cpu_requested;     /* Σ requested cpu over nodes after the run */
  int64_t mem_requested;
} ksg_replica_summary;

typedef struct ksg_ctx ksg_ctx;

int ksg_abi_version(void);
/* sha256 (hex) of the sources the library was built from (csrc/, include/),
 * embedded at build time; bench.py and the tests compare it with the tree. */
const char* ksg_source_hash(void);
int ksg_open(int device, ksg_ctx** out);
int ksg_close(ksg_ctx* ctx);
const char* ksg_last_error(ksg_ctx* ctx);

int ksg_set_profile(ksg_ctx* ctx, const ksg_profile* prof);
int ksg_load_nodes(ksg_ctx* ctx, const ksg_nodes* nodes, const ksg_topology* topo);
int ksg_load_workload(ksg_ctx* ctx, const ksg_workload* wl);

/* Append pods to the loaded workload (the scheduler's per-cycle path: a new
 * pod is encoded against the loaded universe and appended; include/
 * ksched_snapshot.h does both).  tail->pods' program offsets are absolute in
 * the pool; tail->prog holds pool words [prog_base, prog_base +
 * tail->prog_len), and prog_base must not cut into a program an earlier pod
 * uses.  The new pods get indices n_pods, n_pods + 1, ... */
int ksg_append_pods(ksg_ctx* ctx, const ksg_workload* tail, int64_t prog_base);
/* Evaluate pod `pod` (index into the loaded workload) against the current
 * node state; no state change.  `cap` may be NULL.  A pod whose plugins are
 * all node-local takes the chip-wide per-cycle path (one cooperative launch
 * writing into a pinned host block, completion polled from a flag there,
 * persistent buffers); a PodTopologySpread / InterPodAffinity pod takes the
 * chip-wide topology kernel in its evaluate-only capture form, also writing
 * into the pinned block. */
int ksg_eval(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap);

/* The per-cycle results of ksg_eval_view, in library memory (no copy into
 * caller arrays): valid until the next ksg_eval / ksg_eval_view / ksg_eval_pod
 * on the context.  Rows hold elem_bytes-wide integers, one per node: 1 =
 * unsigned byte (the node-local per-cycle path when every raw score is in
 * [0, 255]), else signed (2 when every raw score, normalised score and
 * weighted total fits 16 bits, 4 when they fit 32 bits, else 8); raw[pl] / norm[pl] are
 * NULL for a plugin the profile does not score (norm[pl] == raw[pl] for the
 * plugins without ScoreExtensions).  A pod with fewer than two feasible nodes
 * has all-zero rows (no Score runs).  The Go shim's Score / NormalizeScore
 * answers read these rows directly (wrappedplugin.go:420-445 / 388-415). */
typedef struct ksg_eval_rows {
  int32_t n_nodes;
  int32_t elem_bytes;
  const uint32_t* fstatus;                /* [n_nodes] Filter status words */
  const void* raw[KSG_NPLUGINS];
  const void* norm[KSG_NPLUGINS];         /* NULL for a plugin in norm_from_raw */
  const void* total;                      /* [n_nodes] weighted totals (0: not scored); NULL when the
                                           * evaluation did not materialise them (the node-local per-cycle
                                           * kernel: the framework sums the weights itself) */
  /* Normalised rows the caller derives (round 6: the node-local per-cycle
   * kernel no longer stores them): for plugin p in norm_from_raw, at a
   * feasible node of a scored pod (p in norm_scored), DefaultNormalizeScore
   * of raw[p] with the maximum norm_max[p] over the feasible nodes:
   * TaintToleration (reverse) max ? 100 - 100 * raw / max : 100,
   * NodeAffinity max ? 100 * raw / max : raw (integer division); 0 elsewhere. */
  uint32_t norm_from_raw;
  uint32_t norm_scored;
  int64_t norm_max[KSG_NPLUGINS];
} ksg_eval_rows;
/* ksg_eval with the rows left in library memory (the per-cycle call of the Go
 * shim; replaces the framework's per-(pod, node, plugin) Filter / Score /
 * NormalizeScore calls, wrappedplugin.go:388-548). */
int ksg_eval_view(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_eval_rows* rows);
/* Evaluate an encoded pod that is not part of the workload: `pod`'s program
 * offsets index `prog[0 .. prog_len)`.  Same outputs as ksg_eval; the pod
 * is not retained (ksg_append_pods it first to commit it). */
int ksg_eval_pod(ksg_ctx* ctx, const ksg_pod* pod, const int32_t* prog, int64_t prog_len, ksg_result* res,
                 ksg_capture* cap);
/* Assume pod `pod` onto node `node` (NodeInfo.AddPod + count tables).
 * Stream-ordered: returns once the update is enqueued; every later
 * evaluation and read-back of the context sees it. */
int ksg_commit(ksg_ctx* ctx, int32_t pod, int32_t node);
/* NodeInfo.AddPod of n pods at once: pods[i] onto nodes[i] (the pods already
 * running when a snapshot is loaded, NodeInfo.Pods; the snapshot's replay of
 * its bindings).  One launch, one lane per pod, every update an atomic
 * addition (the result does not depend on the order of the AddPod calls). */
int ksg_commit_batch(ksg_ctx* ctx, const int32_t* pods, const int32_t* nodes, int32_t n);
/* Schedule pods [first, first+count) in order on the device.  placements
 * [count]; results [count] may be NULL; cap may be NULL (else per-pod arrays
 * of count * n_nodes entries). */
int ksg_run_queue(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements,
                  ksg_result* results, ksg_capture* cap);
/* What-if replicas: each replica starts from the loaded node state, uses its
 * own profile and schedules the same pods [first, first+count).
 * placements [n_replicas][count]; summaries [n_replicas] may be NULL. */
int ksg_run_replicas(ksg_ctx* ctx, const ksg_profile* profiles, int32_t n_replicas,
                     int32_t first, int32_t count, int32_t* placements,
                     ksg_replica_summary* summaries);
int ksg_read_state(ksg_ctx* ctx, ksg_node_state* out);

/* ---- DefaultPreemption PostFilter (wrappedplugin.go:550-583 wraps it; the
 * plugin itself is upstream v1.32 defaultpreemption/default_preemption.go,
 * not vendored) ------------------------------------------------------------ */
/* SelectVictimsOnNode for n_cand candidate nodes at once, on the current
 * node state.  Candidate k is node cand_node[k]; its potential victims (the
 * pods on it with lower priority than `pod`, most important first:
 * util.MoreImportantPod order) are vic_pod[vic_off[k] .. vic_off[k+1]).
 * Per candidate: remove every potential victim, re-run the filters that read
 * the node's pods for `pod` (NodeResourcesFit; NodePorts on the UsedPorts
 * the removals leave; PodTopologySpread and InterPodAffinity with the
 * PreFilter counts of the candidate's domains moved by the removals, as the
 * RemovePod / AddPod extensions move them upstream)
 * (fits[k] = 0: the node cannot help), then reprieve the victims in order,
 * each staying evicted (victim[i] = 1) only if `pod` no longer fits with it
 * back.  Node-static filters are not re-run: the caller drops the nodes
 * whose static filters reject `pod` first (ksg_eval_skipping below).
 * KSG_E_UNSUPPORTED when the preemptor's terms exceed the dry run's limits. */
int ksg_preempt_victims(ksg_ctx* ctx, int32_t pod, const int32_t* cand_node, int32_t n_cand,
                        const int32_t* vic_off, const int32_t* vic_pod, int32_t* fits, uint8_t* victim);
/* ksg_eval of loaded pod `pod` with the Filter plugins in `filter_skip`
 * (bit = plugin id) skipped as a PreFilter Skip would skip them; the pod's
 * record is restored before the call returns.  DefaultPreemption asks it
 * with the four pod-dependent filters skipped: a node whose status word is
 * then 0 passes every node-static filter (VolumeBinding, VolumeZone, ...
 * ordered after NodeResourcesFit included), the part of
 * SelectVictimsOnNode's RunFilterPluginsWithNominatedPods (upstream v1.32
 * preemption.go, called from default_preemption.go:SelectVictimsOnNode) no
 * removal can change. */
int ksg_eval_skipping(ksg_ctx* ctx, int32_t pod, uint32_t filter_skip, ksg_result* res, ksg_capture* cap);
/* A victim's deletion: the inverse of ksg_commit (NodeInfo.RemovePod and the
 * count tables), applied by DefaultPreemption's prepareCandidate. */
int ksg_uncommit(ksg_ctx* ctx, int32_t pod, int32_t node);

/* Restore the node state captured at the last ksg_load_nodes(). */
int ksg_reset_state(ksg_ctx* ctx);
/* Timing of the last ksg_run_queue / ksg_run_replicas kernel: milliseconds
 * between HIP events recorded on the stream the kernel was launched on. */
int ksg_last_kernel_ms(ksg_ctx* ctx, double* ms);
/* Which path the last ksg_run_queue / ksg_run_replicas / ksg_eval took: path
 * 1 queue kernel, 2 batched, 3 replica sweep, 4 chip-wide topology, 5 the
 * per-cycle chip-wide evaluation of ksg_eval, 6 its topology form (a
 * PodTopologySpread / InterPodAffinity pod on the chip-wide topology kernel,
 * no assume); flags: the range-
 * checked narrow forms that ran (exact either way; for tests and reports). */
#define KSG_RUN_NARROW_SWEEP 1   /* replica sweep on the 16-byte records */
#define KSG_RUN_SLOT32 2         /* slot walk with 32-bit Fit / BalancedAllocation */
/* 4: the transposed walk (KSG_RUN_TCOL, retired in ABI 4) */
#define KSG_RUN_SPEC 8           /* phase 2 was the speculate-and-verify walk (ksg_batch_phase2v) */
#define KSG_RUN_WIDE_MEM 16      /* ... in its wide-memory instance (memory not whole MiB: int64 bytes) */
#define KSG_RUN_TOPO_WINDOW 32   /* path 4 ran the speculative topology queue (window rows + walk) */
int ksg_last_run_info(ksg_ctx* ctx, int32_t* path, int32_t* flags);

/* Grid-barrier timeouts this context recovered from since it opened.  The
 * chip-wide topology path, the multi-workgroup replica sweep and the
 * per-cycle kernels launch plainly with a grid inside the occupancy API's
 * co-resident count and bound their barrier polls; a timeout (a workgroup was
 * not resident) restores the node state the call started from (a topology
 * queue's partial commits included), switches the context to cooperative
 * launches and runs the same call again, so the caller sees the exact
 * result.  A timeout under a cooperative launch is KSG_E_DEVICE.  (No
 * reference counterpart: device residency.) */
int ksg_recoveries(ksg_ctx* ctx, int32_t* n);

/* The last placement run's speculative topology queue (KSG_RUN_TOPO_WINDOW):
 * windows walked, pods decided, windows a changed node ended early.  All 0
 * when the run took another path.  (No reference counterpart: the reference
 * schedules one pod per cycle.) */
int ksg_topo_window_stats(ksg_ctx* ctx, int64_t* windows, int64_t* pods, int64_t* cut);

/* Per-kernel timing of the next runs (off by default: it adds one event
 * record per launch).  With timing on, ksg_kernel_stats() returns, per kernel
 * that ran in the last ksg_run_queue / ksg_run_replicas call, the number of
 * launches, the summed launch durations (HIP events on the launch stream,
 * between consecutive launches) and the algorithmic units processed:
 * (pod, node) pairs for the sweeping kernels; for the top-set phase 2,
 * Σ_j (j + 1) = top-set entries + changed-node records of a batch.
 * *n = number of kernels (may exceed max). */
enum {
  KSG_K_QUEUE = 0,
  KSG_K_QUEUE_TOPO = 1,
  KSG_K_BATCH_PHASE1 = 2,
  KSG_K_BATCH_TOPK = 3,
  KSG_K_BATCH_PHASE2S = 4,
  KSG_K_SWEEP_STATIC = 5,
  KSG_K_SWEEP = 6,
  KSG_K_TOPO_COOP = 7,
  KSG_K_SWEEP_NARROW = 8,
  KSG_K_CAPTURE_EVAL = 9,
  KSG_K_CAPTURE_NORM = 10,
  KSG_K_EVAL_CYCLE = 11,
  KSG_K_BATCH_PHASE2V = 12,
  KSG_K_TOPO_WIN_ROWS = 13,   /* the window rows (walk included: the last workgroup decides) */
  KSG_NKERNELS = 14
};
typedef struct ksg_kernel_stat {
  char name[48];
  int32_t kind;      /* KSG_K_* */
  int32_t calls;
  double total_ms;
  double units;      /* (pod, node) pairs processed over all launches */
} ksg_kernel_stat;
int ksg_set_timing(ksg_ctx* ctx, int on);
int ksg_kernel_stats(ksg_ctx* ctx, ksg_kernel_stat* out, int32_t max, int32_t* n);

/* ---- bulk result-store serialiser (host code; no device needed) ---------
 * Emits the filter-result, score-result and finalscore-result annotation
 * values of one pod straight from its capture SoA, byte-identical to
 * resultstore.Store.GetStoredResult (store.go:133-198) after the wrapped
 * plugins' AddFilterResult (store.go:423), AddScoreResult (:461) and
 * AddNormalizedScoreResult (:481) calls, i.e. Go encoding/json of the maps. */
typedef struct ksg_names {
  int32_t n_nodes;
  const char* const* node;         /* [n_nodes] node names (UTF-8)                    */
  const char* const* plugin;       /* [KSG_NPLUGINS] names the Store keys plugins by  */
  int32_t n_res;
  const char* const* res;          /* [n_res] resource names ("Insufficient <name>")  */
  int32_t n_taint_vocab;
  const char* const* taint;        /* [n_taint_vocab] "{<key>: <value>}"               */
  int32_t max_taints;
  const uint32_t* taints;          /* [max_taints][n_nodes] as in ksg_nodes.taints    */
} ksg_names;

typedef struct ksg_annotate_in {
  int32_t n_filter;
  const int32_t* filter_order;     /* Filter plugins that ran (PreFilter not Skip), in run order */
  int32_t n_score;
  const int32_t* score_order;      /* Score plugins that ran (PreScore not Skip)      */
  uint32_t normalize_mask;         /* bit p: plugin p has ScoreExtensions             */
  const int64_t* weight;           /* [KSG_NPLUGINS] Store score weight (0 = missing) */
  int32_t n_feasible;              /* < 2: no score / finalscore entries              */
  const uint32_t* fstatus;         /* [n_nodes]  one pod's capture (ksg_capture)       */
  const int64_t* raw;              /* [KSG_NPLUGINS][n_nodes]                          */
  const int64_t* norm;             /* [KSG_NPLUGINS][n_nodes]                          */
} ksg_annotate_in;

typedef struct ksg_annotator ksg_annotator;
int ksg_annotator_new(const ksg_names* names, ksg_annotator** out);
int ksg_annotator_free(ksg_annotator* a);
/* json[0..2] / len[0..2]: filter-result, score-result, finalscore-result.  The
 * strings are owned by the annotator and valid until its next call. */
int ksg_annotate(ksg_annotator* a, const ksg_annotate_in* in, const char** json, int64_t* len);

/* ---- the same values serialised on the device (round 5) -----------------
 * ksg_annotator_attach uploads the annotator's escaped pieces (node keys in
 * name order, plugin keys, messages) to the context, with the Store's score
 * weights [KSG_NPLUGINS] and the plugins with ScoreExtensions.  Then
 * ksg_run_queue_json runs ksg_run_queue(first, count) with capture and writes
 * every pod's filter-result, score-result and finalscore-result on the device
 * from the capture rows, byte-identical to ksg_annotate on the same capture:
 * *json = the values back to back (pod k's three at offsets[3k .. 3k + 3]),
 * in context-owned pinned memory.  ksg_run_queue_json_async returns once the
 * values are written on the device, their copy back in flight on a stream
 * of its own, with a ticket for ksg_json_wait; three buffers rotate, so a
 * chunk's values stay valid until the third launch after it (consume chunk i
 * while chunk i + 1 is copied back and chunk i + 2 computed).  Pods the
 * batched / chip-wide capture paths do not take (host ports, claims) are
 * refused (KSG_E_UNSUPPORTED): use ksg_annotate for those. */
int ksg_annotator_attach(ksg_ctx* ctx, const ksg_annotator* a, const int64_t* weight, uint32_t normalize_mask);
int ksg_run_queue_json(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                       const char** json, const int64_t** offsets);
int ksg_run_queue_json_async(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                             int32_t* ticket);
int ksg_json_wait(ksg_ctx* ctx, int32_t ticket, const char** json, const int64_t** offsets);

#ifdef __cplusplus
}
#endif
#endif /* KSCHED_H */
