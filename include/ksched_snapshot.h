/*
 * ksched_snapshot.h — native snapshot encoder of libksched.so (host code).
 *
 * North-star subsystem (1): NodeInfo / PodInfo -> the SoA columns, interned
 * ids and compiled selector programs of ksched.h, built from flat C views of
 * the v1.Node / v1.Pod fields the in-tree Filter/Score plugins read.  A cgo
 * caller fills these views straight from the objects the framework hands to
 * the wrapped plugins:
 *   PreFilter(ctx, state, *v1.Pod)             wrappedplugin.go:491 (-> :504)
 *   Filter(ctx, state, *v1.Pod, *NodeInfo)     wrappedplugin.go:523 (-> :535)
 * and from handle.SnapshotSharedLister().NodeInfos().List() for the node set
 * (INTEGRATION.md §3).  No Python is involved: the encoder, the device
 * library and the status-message decoder are one native library.
 *
 * Views are read during the call only (cgo pointer rules); strings are
 * NUL-terminated UTF-8.  Every function returns 0 or a negative KSG_E_* code;
 * ksg_snapshot_error() gives the message.  A snapshot is not thread-safe.
 *
 * Life cycle:
 *   ksg_snapshot_new(profile)            KubeSchedulerConfiguration profile 0
 *   ksg_snapshot_add_node(...)           every node, in snapshot order
 *   ksg_snapshot_add_pod(...)            every pod that is or will be bound
 *   ksg_snapshot_bind(pod, node)         pods already running (NodeInfo.Pods)
 *   ksg_snapshot_load(ctx)               encode + load into a device context,
 *                                        replaying the bindings
 * then per scheduling cycle:
 *   ksg_snapshot_add_pod(new pod)        -> pod index
 *   ksg_snapshot_sync(ctx)               appends the pod to the device
 *                                        workload when the encoding universe
 *                                        (label columns, value ids, selectors,
 *                                        term templates) is unchanged, else
 *                                        re-encodes and reloads everything
 *   ksg_eval(ctx, pod, ...)              one sweep (ksched.h)
 *   ksg_snapshot_assume(ctx, pod, node)  Reserve: ksg_commit + binding record
 *   ksg_snapshot_status(...)             framework.Status code + message of a
 *                                        node's filter status word
 */
#ifndef KSCHED_SNAPSHOT_H
#define KSCHED_SNAPSHOT_H

#include "ksched.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ksg_str_pair { const char* key; const char* value; } ksg_str_pair;

/* A resource quantity: cpu in millicores (Quantity.MilliValue), every other
 * resource in base units (Quantity.Value).  Also (name, weight) pairs of the
 * plugin args' resource lists. */
typedef struct ksg_quantity { const char* name; int64_t value; } ksg_quantity;

typedef struct ksg_taint_view { const char* key; const char* value; const char* effect; } ksg_taint_view;

/* operator: "" / "Equal" / "Exists"; effect "" = every effect */
typedef struct ksg_toleration_view {
  const char* key;
  const char* op;
  const char* value;
  const char* effect;
} ksg_toleration_view;

/* NodeSelectorRequirement / LabelSelectorRequirement:
 * op "In" "NotIn" "Exists" "DoesNotExist" "Gt" "Lt" */
typedef struct ksg_requirement_view {
  const char* key;
  const char* op;
  int32_t n_values;
  const char* const* values;
} ksg_requirement_view;

typedef struct ksg_node_selector_term_view {
  int32_t n_expr;
  const ksg_requirement_view* expr;     /* matchExpressions */
  int32_t n_fields;
  const ksg_requirement_view* fields;   /* matchFields (metadata.name) */
} ksg_node_selector_term_view;

typedef struct ksg_preferred_term_view {
  int32_t weight;
  ksg_node_selector_term_view preference;
} ksg_preferred_term_view;

/* metav1.LabelSelector; is_set = 0 models a nil pointer */
typedef struct ksg_label_selector_view {
  int32_t is_set;
  int32_t n_labels;
  const ksg_str_pair* match_labels;
  int32_t n_expr;
  const ksg_requirement_view* expr;
} ksg_label_selector_view;

/* PodAffinityTerm (weight: WeightedPodAffinityTerm.weight, preferred terms only) */
typedef struct ksg_affinity_term_view {
  int32_t weight;
  ksg_label_selector_view selector;
  const char* topology_key;
  int32_t n_namespaces;
  const char* const* namespaces;
  ksg_label_selector_view namespace_selector;   /* is_set 0 = nil */
} ksg_affinity_term_view;

/* TopologySpreadConstraint; min_domains 0 = nil; policies NULL/"" = nil */
typedef struct ksg_spread_view {
  int32_t max_skew;
  const char* topology_key;
  const char* when_unsatisfiable;   /* "DoNotSchedule" / "ScheduleAnyway" */
  ksg_label_selector_view selector;
  int32_t min_domains;
  const char* node_affinity_policy;
  const char* node_taints_policy;
  int32_t n_match_label_keys;
  const char* const* match_label_keys;
} ksg_spread_view;

/* One containers[].ports[] entry with a hostPort (v1.ContainerPort): the
 * NodePorts plugin's input (schedutil.GetHostPorts).  host_ip / protocol may
 * be "" or NULL (sanitised to 0.0.0.0 / TCP as HostPortInfo does); entries
 * with host_port <= 0 are ignored. */
typedef struct ksg_host_port_view {
  const char* host_ip;
  const char* protocol;
  int32_t host_port;
  int32_t pad;
} ksg_host_port_view;

typedef struct ksg_container_view {
  const char* image;
  int32_t n_requests;
  const ksg_quantity* requests;
  int32_t restartable;      /* init container with restartPolicy Always (sidecar) */
  int32_t n_host_ports;
  const ksg_host_port_view* host_ports;
} ksg_container_view;

typedef struct ksg_image_view {
  int32_t n_names;
  const char* const* names;
  int64_t size_bytes;
} ksg_image_view;

typedef struct ksg_node_view {
  const char* name;
  int32_t n_labels;
  const ksg_str_pair* labels;
  int32_t n_taints;
  const ksg_taint_view* taints;
  int32_t n_alloc;
  const ksg_quantity* allocatable;   /* status.allocatable, "pods" included */
  int32_t unschedulable;             /* spec.unschedulable */
  int32_t n_images;
  const ksg_image_view* images;      /* status.images */
} ksg_node_view;

/* One spec.volumes[] entry (v1.Volume): kind = the JSON key of the
 * VolumeSource field that is set ("persistentVolumeClaim", "emptyDir",
 * "configMap", ...), claim_name = persistentVolumeClaim.claimName.  A claim
 * makes VolumeBinding / NodeVolumeLimits / VolumeRestrictions / VolumeZone
 * PreFilter run: the claim is resolved against the PersistentVolumeClaims,
 * PersistentVolumes and StorageClasses added with ksg_snapshot_add_pvc /
 * _add_pv / _add_storage_class (their listers), the PreFilter outcomes are
 * decided at encode, the per-node Filter predicates go to the device as the
 * pod's volume program.  A generic ephemeral volume or an in-tree disk volume
 * (gcePersistentDisk, awsElasticBlockStore, azureDisk, azureFile, cinder,
 * vsphereVolume, portworxVolume, rbd, iscsi) is refused (KSG_E_UNSUPPORTED)
 * while a volume plugin is enabled; every other source is their Skip, as
 * upstream. */
typedef struct ksg_volume_view {
  const char* name;
  const char* kind;
  const char* claim_name;
} ksg_volume_view;

/* v1.PersistentVolume as VolumeBinding / VolumeZone read it
 * (simulator/snapshot/snapshot.go:34 pvs). */
typedef struct ksg_pv_view {
  const char* name;
  int32_t n_labels;
  const ksg_str_pair* labels;                /* metadata.labels (VolumeZone) */
  const char* storage_class;                 /* storagehelpers.GetPersistentVolumeClass: the beta
                                                annotation, else spec.storageClassName ("" none) */
  const char* claim_namespace;               /* spec.claimRef (claim_name NULL = no claimRef) */
  const char* claim_name;
  const char* source;                        /* the JSON key of the PersistentVolumeSource set ("csi", ...) */
  int32_t has_node_affinity;                 /* spec.nodeAffinity.required != nil */
  int32_t n_terms;
  const ksg_node_selector_term_view* terms;  /* its nodeSelectorTerms */
} ksg_pv_view;

/* v1.PersistentVolumeClaim (snapshot.go:35 pvcs). */
typedef struct ksg_pvc_view {
  const char* namespace_;
  const char* name;
  const char* volume_name;                   /* spec.volumeName ("" unbound) */
  const char* storage_class;                 /* GetPersistentVolumeClaimClass: the beta annotation,
                                                else spec.storageClassName ("" none) */
  int32_t n_access_modes;
  const char* const* access_modes;           /* spec.accessModes */
  int32_t n_annotations;
  const ksg_str_pair* annotations;           /* bind-completed, selected-node */
  int32_t deleting;                          /* metadata.deletionTimestamp != nil */
} ksg_pvc_view;

/* storagev1.StorageClass (snapshot.go:36 storageClasses), after API
 * defaulting (volumeBindingMode "" = Immediate). */
typedef struct ksg_topology_requirement_view {
  const char* key;
  int32_t n_values;
  const char* const* values;
} ksg_topology_requirement_view;
typedef struct ksg_topology_term_view {
  int32_t n_requirements;
  const ksg_topology_requirement_view* requirements;   /* matchLabelExpressions */
} ksg_topology_term_view;
typedef struct ksg_storage_class_view {
  const char* name;
  const char* provisioner;
  const char* binding_mode;                  /* "Immediate" / "WaitForFirstConsumer" */
  int32_t n_allowed_topologies;
  const ksg_topology_term_view* allowed_topologies;
} ksg_storage_class_view;

typedef struct ksg_pod_view {
  const char* namespace_;
  const char* name;
  int32_t n_labels;
  const ksg_str_pair* labels;
  int32_t n_containers;
  const ksg_container_view* containers;
  int32_t n_init_containers;
  const ksg_container_view* init_containers;
  int32_t has_overhead;
  int32_t n_overhead;
  const ksg_quantity* overhead;
  const char* node_name;                     /* spec.nodeName ("" = unset) */
  int32_t has_node_selector;                 /* spec.nodeSelector != nil */
  int32_t n_node_selector;
  const ksg_str_pair* node_selector;
  int32_t has_na_required;                   /* requiredDuringScheduling... != nil */
  int32_t n_na_required;
  const ksg_node_selector_term_view* na_required;
  int32_t has_na_preferred;                  /* preferredDuringScheduling... != nil */
  int32_t n_na_preferred;
  const ksg_preferred_term_view* na_preferred;
  int32_t n_pod_affinity_required;
  const ksg_affinity_term_view* pod_affinity_required;
  int32_t n_pod_affinity_preferred;
  const ksg_affinity_term_view* pod_affinity_preferred;
  int32_t n_pod_anti_affinity_required;
  const ksg_affinity_term_view* pod_anti_affinity_required;
  int32_t n_pod_anti_affinity_preferred;
  const ksg_affinity_term_view* pod_anti_affinity_preferred;
  int32_t n_tolerations;
  const ksg_toleration_view* tolerations;
  int32_t n_spread;
  const ksg_spread_view* spread;
  /* helper.DefaultSelector over the Services / RCs / RSs / StatefulSets that
   * select the pod (PodTopologySpread system defaults); is_set 0 = none */
  ksg_label_selector_view default_spread_selector;
  int32_t terminating;                       /* metadata.deletionTimestamp != nil */
  int32_t priority;                          /* corev1helpers.PodPriority */
  int32_t n_volumes;
  const ksg_volume_view* volumes;            /* spec.volumes */
} ksg_pod_view;

typedef struct ksg_plugin_view { const char* name; int32_t weight; } ksg_plugin_view;

/* Extension points whose per-point plugin sets the evaluator models. */
#define KSG_POINT_PREFILTER 0
#define KSG_POINT_FILTER 1
#define KSG_POINT_PRESCORE 2
#define KSG_POINT_SCORE 3
#define KSG_NPOINTS 4

/* One extension point's configv1.PluginSet as ConvertForSimulator keeps it
 * (plugins.go:177-186 applyPluginSet: enabled plugins renamed to XWrapped with
 * their weights, disabled ones renamed except "*"; either spelling is
 * accepted).  n_enabled = n_disabled = 0: the point is not configured and
 * takes the MultiPoint expansion alone. */
typedef struct ksg_plugin_set_view {
  int32_t n_enabled;
  const ksg_plugin_view* enabled;
  int32_t n_disabled;
  const char* const* disabled;
} ksg_plugin_set_view;

/* Profile 0 after ConvertForSimulator (plugins.go:174-197): MultiPoint plugins
 * in order (names with or without the "Wrapped" suffix), weights as written
 * (getScorePluginWeight maps 0 to 1, plugins.go:289-304), the per-point sets
 * (PreFilter / Filter / PreScore / Score), and the plugin args the evaluator
 * models, as the plugin factories receive them decoded (defaults:
 * plugins_test.go:876-1000). */
typedef struct ksg_profile_view {
  int32_t n_plugins;
  const ksg_plugin_view* plugins;
  const char* fit_strategy;                  /* "LeastAllocated" / "MostAllocated" /
                                                "RequestedToCapacityRatio" (shape below) */
  int32_t n_fit_resources;
  const ksg_quantity* fit_resources;         /* (name, weight) */
  int32_t n_ba_resources;
  const ksg_quantity* ba_resources;
  int32_t n_fit_ignored_resources;
  const char* const* fit_ignored_resources;
  int32_t n_fit_ignored_groups;
  const char* const* fit_ignored_groups;
  int32_t hard_pod_affinity_weight;
  int32_t ignore_preferred_terms_of_existing_pods;
  int32_t pts_system_defaulted;              /* PodTopologySpreadArgs.defaultingType == System */
  int32_t ba_skip_best_effort;
  ksg_plugin_set_view points[KSG_NPOINTS];   /* indexed by KSG_POINT_* */
  /* NodeResourcesFitArgs.scoringStrategy.requestedToCapacityRatio.shape as
   * written (utilization 0..100 increasing, score 0..10; at most
   * KSG_MAX_SHAPE points), read when fit_strategy is RequestedToCapacityRatio */
  int32_t n_shape;
  const int32_t* shape_utilization;
  const int32_t* shape_score;
  /* PodTopologySpreadArgs.defaultConstraints (defaultingType List, i.e.
   * pts_system_defaulted = 0): selector unset, the owners' selector is used */
  int32_t n_default_constraints;
  const ksg_spread_view* default_constraints;
} ksg_profile_view;

/* The profile as the framework and the simulator's Store see it (derived by
 * ksg_snapshot_new from ksg_profile_view):
 *   order[KSG_POINT_*]  plugin ids each extension point runs, in order: the
 *                       framework's expansion of MultiPoint into the point
 *                       [upstream v1.32 expandMultiPointPlugins, TO VERIFY:
 *                       DESIGN.md §9]: the point's own plugins that
 *                       MultiPoint also lists, then the other MultiPoint
 *                       plugins implementing the point and not disabled
 *                       there, then the point's remaining plugins;
 *   store_weight        getScorePluginWeight (plugins.go:289-304): Score
 *                       enabled then MultiPoint enabled, a later entry
 *                       replaces an earlier one, 0 -> 1; 0 = not in the map
 *                       (the Store then records final = raw x 0).  This is
 *                       the weight array ksg_annotate takes;
 *   selection_weight    the framework's weight of each Score plugin in the
 *                       weighted total (the point's own weight first);
 *   normalize_mask      plugins with ScoreExtensions. */
typedef struct ksg_profile_info {
  int32_t n_order[KSG_NPOINTS];
  int32_t order[KSG_NPOINTS][KSG_NPLUGINS];
  int64_t store_weight[KSG_NPLUGINS];
  int32_t selection_weight[KSG_NPLUGINS];
  uint32_t normalize_mask;
  int32_t pad;
} ksg_profile_info;

typedef struct ksg_snapshot ksg_snapshot;

/* framework.Code values used by ksg_snapshot_status */
#define KSG_CODE_SUCCESS 0
#define KSG_CODE_UNSCHEDULABLE 2
#define KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE 3
#define KSG_CODE_SKIP 5

int ksg_snapshot_new(const ksg_profile_view* profile, ksg_snapshot** out);
/* The derived extension-point orders and the two weight maps (no device). */
int ksg_snapshot_profile_info(ksg_snapshot* s, ksg_profile_info* out);
int ksg_snapshot_free(ksg_snapshot* s);
const char* ksg_snapshot_error(ksg_snapshot* s);

int ksg_snapshot_add_node(ksg_snapshot* s, const ksg_node_view* node, int32_t* index);
int ksg_snapshot_add_pod(ksg_snapshot* s, const ksg_pod_view* pod, int32_t* index);
/* Namespace `name` with its labels (v1.Namespace; the exported snapshot's
 * namespaces).  Pod (anti-)affinity terms whose namespaceSelector has
 * requirements resolve against the namespaces added so far, as the
 * InterPodAffinity PreFilter's namespace lister would
 * (mergeAffinityTermNamespacesIfNotEmpty): namespaces ∪ {matching names}.
 * A pod with such a term is refused (KSG_E_UNSUPPORTED) until at least one
 * namespace was added; adding or relabelling a namespace re-resolves every
 * pod's terms (the next sync re-encodes when any changed).  Replaces the
 * reference's namespace informer feed (snapshot.go namespaces). */
int ksg_snapshot_add_namespace(ksg_snapshot* s, const char* name, int32_t n_labels, const ksg_str_pair* labels);
/* The volume plugins' listers (snapshot.go:34-36): a PersistentVolume,
 * PersistentVolumeClaim or StorageClass added or replaced (same name) is read
 * by the next encode, which is a full one (every pod's claims resolve again).
 * A node publishing CSI attach limits (allocatable attachable-volumes-csi-*)
 * with NodeVolumeLimits enabled and a pod with claims is refused at encode. */
int ksg_snapshot_add_pv(ksg_snapshot* s, const ksg_pv_view* pv);
int ksg_snapshot_add_pvc(ksg_snapshot* s, const ksg_pvc_view* pvc);
int ksg_snapshot_add_storage_class(ksg_snapshot* s, const ksg_storage_class_view* sc);
/* Drops every PersistentVolume, claim and StorageClass (the listers' state
 * before a resync: the Go shim clears, then re-adds what its listers hold, so
 * a deleted object leaves the snapshot and a pod naming a deleted claim is
 * rejected at PreFilter as upstream's lister lookup would reject it).  The
 * next encode is a full one when anything was dropped. */
int ksg_snapshot_clear_storage(ksg_snapshot* s);
/* A pod the caller will add later (a pending pod of the scheduling queue, as
 * the pod informer delivers it: upstream eventhandlers.go addPodToSchedulingQueue
 * feeding the simulator's scheduler).  Its selectors, term templates, label
 * keys, scalar resources and host ports join the encoding universe at the
 * next encode / sync: that sync re-encodes only when a hint brings in
 * something the current encoding lacks (each new hint is encoded against the
 * frozen universe first, as an append would be), once per batch of such hints;
 * the pod itself is not a workload pod until ksg_snapshot_add_pod, which also
 * drops its hint (matched by namespace and name).  Adding it then appends in
 * place (ksg_snapshot_sync *appended = 1) instead of re-encoding.  Hints never
 * change a result: a selector or template nobody evaluates is only data. */
int ksg_snapshot_hint_pod(ksg_snapshot* s, const ksg_pod_view* pod);
/* A hinted pod was deleted before it was added (the informer's delete of a
 * pending pod, upstream eventhandlers.go deletePodFromSchedulingQueue): its
 * hint is dropped.  Namespace null = "default".  Unknown pods are ignored. */
int ksg_snapshot_unhint_pod(ksg_snapshot* s, const char* namespace_, const char* name);
/* Pod `pod` runs on `node` (NodeInfo.Pods): replayed as an assume at load. */
int ksg_snapshot_bind(ksg_snapshot* s, int32_t pod, int32_t node);
int ksg_snapshot_node_index(ksg_snapshot* s, const char* name, int32_t* index);

/* Encode everything added so far (no device needed).  The views below point
 * into the snapshot and stay valid until the next add / encode / sync. */
int ksg_snapshot_encode(ksg_snapshot* s);
int ksg_snapshot_view(ksg_snapshot* s, ksg_nodes* nodes, ksg_topology* topo, ksg_workload* workload,
                      ksg_profile* profile);

/* Encode only the pods added since the last encode: *appended = 1 when none
 * of them extends the encoding universe (they are encoded against it,
 * byte-identical to a full re-encode), 0 when a full re-encode ran. */
int ksg_snapshot_encode_incremental(ksg_snapshot* s, int32_t* appended);

/* Encode, ksg_set_profile + ksg_load_nodes + ksg_load_workload into `ctx`,
 * then replay every binding / assume in order (ksg_commit). */
int ksg_snapshot_load(ksg_snapshot* s, ksg_ctx* ctx);
/* Bring `ctx` up to date after ksg_snapshot_add_pod: *appended = 1 when the new
 * pods were appended (ksg_append_pods), 0 when a full reload was needed. */
int ksg_snapshot_sync(ksg_snapshot* s, ksg_ctx* ctx, int32_t* appended);
/* Reserve / assume: ksg_commit on the device and a binding record (replayed
 * by a later reload). */
int ksg_snapshot_assume(ksg_snapshot* s, ksg_ctx* ctx, int32_t pod, int32_t node);
/* The inverse (a preemption victim's deletion): ksg_uncommit + record. */
int ksg_snapshot_forget(ksg_snapshot* s, ksg_ctx* ctx, int32_t pod, int32_t node);

/* framework.Status of `pod`'s Filter at `node` from its status word
 * (ksg_capture.fstatus): *code = KSG_CODE_*, msg = Status.Message() (reasons
 * joined with ", "), NUL-terminated, truncated to cap - 1 bytes; *len = full
 * length.  Word 0 = Success (empty message). */
int ksg_snapshot_status(ksg_snapshot* s, int32_t pod, uint32_t word, int32_t node, int32_t* code, char* msg,
                        int32_t cap, int32_t* len);
/* Every node's Filter status at once (the Go shim decodes a pod's statuses
 * once per cycle, in evalPod, instead of once per Filter call under a lock):
 * code[n] = KSG_CODE_*, msg[n] = index of the node's Status.Message() among
 * the pod's distinct messages (-1: success or not evaluated).  The distinct
 * messages go to buf NUL-separated in index order when cap >= *len; *n_msgs
 * and *len (bytes, NULs included) are always set, so a caller can size buf
 * and call again. */
int ksg_snapshot_statuses(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes, int32_t* code,
                          int32_t* msg, char* buf, int64_t cap, int32_t* n_msgs, int64_t* len);
/* ksg_snapshot_statuses into arrays the snapshot owns (the per-cycle form;
 * replaces round 5's ksg_snapshot_statuses_delta, which recognised the
 * caller's kept arrays by their addresses): *code / *msg point at n_nodes
 * entries, read-only to the caller, valid until the next
 * ksg_snapshot_statuses_kept call on this snapshot or ksg_snapshot_free.
 * After a complete call they hold exactly its output, so the next call
 * resets only the nodes that call rejected and writes only its own rejected
 * nodes (no pass over the passing nodes); it writes every node when the last
 * call failed, n_nodes changed, or the last call rejected more than an eighth
 * of the nodes.  buf / cap / *n_msgs / *len as ksg_snapshot_statuses.  A
 * caller that retains the statuses past the next cycle copies them. */
int ksg_snapshot_statuses_kept(ksg_snapshot* s, int32_t pod, const uint32_t* words, int32_t n_nodes,
                               const int32_t** code, const int32_t** msg, char* buf, int64_t cap, int32_t* n_msgs,
                               int64_t* len);
/* Calls of ksg_snapshot_statuses_kept that took the sparse / the dense form
 * (diagnostics and tests). */
int ksg_snapshot_statuses_kept_stats(ksg_snapshot* s, int64_t* sparse_calls, int64_t* dense_calls);
/* PreFilter of plugin `plugin` for `pod` (given the device result's status
 * bits): *code = KSG_CODE_SUCCESS / SKIP / UNSCHEDULABLE_AND_UNRESOLVABLE
 * (NodeAffinity "pod affinity terms conflict", a volume plugin's claim /
 * volume lookup: ksg_snapshot_prefilter_message); the PreFilterResult node
 * names (sorted) of NodeAffinity or VolumeBinding go to names[0..*n_names)
 * when *has_result = 1 (names may be NULL to query the count).  The plugins
 * after a rejecting one in the profile's PreFilter order are not run by the
 * framework; an empty intersection of the results is the framework's own
 * rejection (every node is then left unevaluated on the device). */
int ksg_snapshot_prefilter(ksg_snapshot* s, int32_t pod, int32_t plugin, uint32_t result_status, int32_t* code,
                           int32_t* has_result, const char** names, int32_t cap, int32_t* n_names);
/* The PreFilter rejection message of `plugin` for `pod` (the status
 * ksg_snapshot_prefilter returned as KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE:
 * NodeAffinity "pod affinity terms conflict", VolumeRestrictions / VolumeBinding
 * / VolumeZone claim and volume lookups), NUL-terminated, truncated to cap - 1
 * bytes; *len = full length, 0 when the plugin did not reject.  VolumeBinding's
 * PreFilterResult (the nodes of the pod's bound local volumes) comes through
 * ksg_snapshot_prefilter like NodeAffinity's. */
int ksg_snapshot_prefilter_message(ksg_snapshot* s, int32_t pod, int32_t plugin, char* msg, int32_t cap,
                                   int32_t* len);

/* Decode tables of the current encoding (for ksg_annotator_new): node names,
 * resource column names, taint strings "{key: value}". */
int ksg_snapshot_counts(ksg_snapshot* s, int32_t* n_nodes, int32_t* n_pods, int32_t* n_res, int32_t* n_taint_vocab);
int ksg_snapshot_names(ksg_snapshot* s, const char** node, const char** res, const char** taint);

#ifdef __cplusplus
}
#endif
#endif /* KSCHED_SNAPSHOT_H */
