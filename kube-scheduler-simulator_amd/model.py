"""Cluster object model for the Filter/Score path.

This is the host-side view of the objects the upstream plugins read: the
subset of `v1.Node`, `v1.Pod` and `framework.NodeInfo` that the in-tree
Filter/Score plugins of kube-scheduler v1.32 consult.
The simulator hands these objects to the wrapped plugins at
`simulator/scheduler/plugin/wrappedplugin.go:523` (Filter, `*framework.NodeInfo`)
and `:420` (Score, node name).  The snapshot encoder (`encoder.py`) turns a
list of these into the SoA columns the HIP kernels read.

Resource quantities are plain Python ints: cpu in millicores (what
`Quantity.MilliValue()` returns), everything else in base units
(`Quantity.Value()`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

# ---- resource names (k8s.io/api core/v1) ----------------------------------
CPU = "cpu"
MEMORY = "memory"
EPHEMERAL = "ephemeral-storage"
PODS = "pods"

# schedutil.DefaultMilliCPURequest / DefaultMemoryRequest [upstream
# pkg/scheduler/util/pod_resources.go]: applied per container lacking a request
# when computing "non-zero" requests.
DEFAULT_MILLI_CPU_REQUEST = 100
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024

# ---- taint effects / toleration operators ---------------------------------
NO_SCHEDULE = "NoSchedule"
PREFER_NO_SCHEDULE = "PreferNoSchedule"
NO_EXECUTE = "NoExecute"
EFFECTS = (NO_SCHEDULE, PREFER_NO_SCHEDULE, NO_EXECUTE)

OP_EQUAL = "Equal"
OP_EXISTS = "Exists"

# node selector / label selector operators
IN, NOT_IN, EXISTS, DOES_NOT_EXIST, GT, LT = "In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"

LABEL_HOSTNAME = "kubernetes.io/hostname"
LABEL_ZONE = "topology.kubernetes.io/zone"
LABEL_REGION = "topology.kubernetes.io/region"
TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"
OBJECT_NAME_FIELD = "metadata.name"

DO_NOT_SCHEDULE = "DoNotSchedule"
SCHEDULE_ANYWAY = "ScheduleAnyway"
POLICY_HONOR = "Honor"
POLICY_IGNORE = "Ignore"


def is_scalar_resource(name: str) -> bool:
    """schedutil.IsScalarResourceName [upstream]: extended resources
    (a domain-prefixed name outside kubernetes.io/), hugepages-*, and
    attachable-volumes-*."""
    if name.startswith("hugepages-") or name.startswith("attachable-volumes-"):
        return True
    if "/" in name and not name.startswith("kubernetes.io/") and not name.startswith("requests."):
        return True
    return False


@dataclass(frozen=True)
class Taint:
    key: str
    value: str = ""
    effect: str = NO_SCHEDULE


@dataclass(frozen=True)
class Toleration:
    key: str = ""
    operator: str = ""          # "" means Equal
    value: str = ""
    effect: str = ""            # "" means all effects

    def tolerates(self, taint: Taint) -> bool:
        """v1.Toleration.ToleratesTaint [upstream k8s.io/api core/v1/toleration.go]."""
        if self.effect and self.effect != taint.effect:
            return False
        if self.key and self.key != taint.key:
            return False
        if self.operator in ("", OP_EQUAL):
            return self.value == taint.value
        if self.operator == OP_EXISTS:
            return True
        return False


def tolerations_tolerate(tols, taint: Taint) -> bool:
    """v1helper.TolerationsTolerateTaint."""
    return any(t.tolerates(taint) for t in tols)


@dataclass(frozen=True)
class Requirement:
    """A NodeSelectorRequirement or a LabelSelectorRequirement."""
    key: str
    operator: str
    values: Tuple[str, ...] = ()


@dataclass(frozen=True)
class NodeSelectorTerm:
    match_expressions: Tuple[Requirement, ...] = ()
    match_fields: Tuple[Requirement, ...] = ()


@dataclass(frozen=True)
class PreferredSchedulingTerm:
    weight: int
    preference: NodeSelectorTerm


@dataclass(frozen=True)
class LabelSelector:
    """metav1.LabelSelector. `None` (nil) selectors are modelled by the caller."""
    match_labels: Tuple[Tuple[str, str], ...] = ()
    match_expressions: Tuple[Requirement, ...] = ()

    def empty(self) -> bool:
        return not self.match_labels and not self.match_expressions


@dataclass(frozen=True)
class PodAffinityTerm:
    label_selector: Optional[LabelSelector]
    topology_key: str
    namespaces: Tuple[str, ...] = ()
    # None = nil namespaceSelector (matches no namespace); an empty LabelSelector
    # matches every namespace.
    namespace_selector: Optional[LabelSelector] = None


@dataclass(frozen=True)
class WeightedPodAffinityTerm:
    weight: int
    term: PodAffinityTerm


@dataclass(frozen=True)
class TopologySpreadConstraint:
    max_skew: int
    topology_key: str
    when_unsatisfiable: str
    label_selector: Optional[LabelSelector]
    min_domains: Optional[int] = None
    node_affinity_policy: Optional[str] = None
    node_taints_policy: Optional[str] = None
    match_label_keys: Tuple[str, ...] = ()


@dataclass
class Container:
    image: str = ""
    requests: Dict[str, int] = field(default_factory=dict)
    # restartPolicy: Always on an init container makes it a sidecar
    restartable: bool = False
    host_ports: Tuple[Tuple[str, str, int], ...] = ()   # (hostIP, protocol, hostPort)


@dataclass
class Pod:
    name: str
    namespace: str = "default"
    labels: Dict[str, str] = field(default_factory=dict)
    containers: List[Container] = field(default_factory=list)
    init_containers: List[Container] = field(default_factory=list)
    overhead: Optional[Dict[str, int]] = None
    node_name: str = ""
    node_selector: Optional[Dict[str, str]] = None
    # NodeAffinity: None = nil
    node_affinity_required: Optional[List[NodeSelectorTerm]] = None
    node_affinity_preferred: Optional[List[PreferredSchedulingTerm]] = None
    # InterPodAffinity
    pod_affinity_required: List[PodAffinityTerm] = field(default_factory=list)
    pod_affinity_preferred: List[WeightedPodAffinityTerm] = field(default_factory=list)
    pod_anti_affinity_required: List[PodAffinityTerm] = field(default_factory=list)
    pod_anti_affinity_preferred: List[WeightedPodAffinityTerm] = field(default_factory=list)
    tolerations: List[Toleration] = field(default_factory=list)
    topology_spread_constraints: List[TopologySpreadConstraint] = field(default_factory=list)
    # Selector that helper.DefaultSelector would build from the services /
    # RCs / RSs / StatefulSets selecting this pod (PodTopologySpread system
    # default constraints).  None = no such owner/service.
    default_spread_selector: Optional[LabelSelector] = None
    terminating: bool = False
    # DefaultPreemption inputs: corev1helpers.PodPriority (spec.priority, 0
    # when unset), spec.preemptionPolicy ("Never" or "PreemptLowerPriority")
    # and status.startTime in Unix ns (None: not started, util.GetPodStartTime
    # then answers "now", later than every recorded start).
    priority: int = 0
    preemption_policy: str = "PreemptLowerPriority"
    start_time: Optional[int] = None
    # spec.volumes: (name, the v1.VolumeSource field that is set, its JSON key,
    # persistentVolumeClaim.claimName or "")
    volumes: List[Tuple[str, str, str]] = field(default_factory=list)
    # the cluster's PersistentVolumes / claims / StorageClasses, which the
    # volume plugins' listers read for this pod's claims (None: none exist)
    storage: Optional["Storage"] = None

    def claim_names(self) -> List[str]:
        """spec.volumes[].persistentVolumeClaim.claimName, in volume order."""
        return [c for _, k, c in self.volumes if k == "persistentVolumeClaim"]

    def volumes_needing_plugins(self):
        """The volumes whose source makes a volume plugin's PreFilter run
        instead of returning Skip [upstream v1.32 plugins/volumebinding
        (podHasPVCs: claims and generic ephemeral volumes),
        nodevolumelimits/csi.go PreFilter (claims, ephemeral, in-tree volumes
        CSI migration translates), volumerestrictions (GCE PD, AWS EBS, RBD,
        iSCSI, ReadWriteOncePod claims), volumezone (claims)] and that the
        evaluator does not model: generic ephemeral and in-tree disk volumes
        are refused (NotImplementedError) rather than recorded as a Skip
        upstream would not return.  Claims (persistentVolumeClaim) are
        modelled (encoder.py Encoder._volume_plan)."""
        return [(n, k) for n, k, _ in self.volumes if k in VOLUME_SOURCES_REFUSED]

    def has_pod_affinity(self) -> bool:
        return bool(self.pod_affinity_required or self.pod_affinity_preferred
                    or self.pod_anti_affinity_required or self.pod_anti_affinity_preferred)

    def host_ports(self):
        """schedutil.GetHostPorts [upstream v1.32 pkg/scheduler/util, TO
        VERIFY: DESIGN.md §9]: the ports with a hostPort of the init
        containers that keep running (restartPolicy Always, sidecars), then of
        the regular containers, as (hostIP, protocol, hostPort) unsanitised."""
        out = []
        for c in self.init_containers:
            if c.restartable:
                out.extend(x for x in c.host_ports if x[2] > 0)
        for c in self.containers:
            out.extend(x for x in c.host_ports if x[2] > 0)
        return out


VOLUME_SOURCES_REFUSED = frozenset((
    "ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "azureFile",
    "cinder", "vsphereVolume", "portworxVolume", "rbd", "iscsi"))

# ---- storage: what VolumeBinding / VolumeZone / VolumeRestrictions /
# NodeVolumeLimits read through their listers [upstream v1.32
# pkg/scheduler/framework/plugins/{volumebinding,volumezone,volumerestrictions,
# nodevolumelimits}; k8s.io/api storage/v1, core/v1 — not vendored]
READ_WRITE_ONCE_POD = "ReadWriteOncePod"
BINDING_IMMEDIATE = "Immediate"
BINDING_WAIT_FOR_FIRST_CONSUMER = "WaitForFirstConsumer"
NOT_SUPPORTED_PROVISIONER = "kubernetes.io/no-provisioner"
ANN_BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
ANN_SELECTED_NODE = "volume.kubernetes.io/selected-node"
ANN_BETA_STORAGE_CLASS = "volume.beta.kubernetes.io/storage-class"
# volumezone.topologyLabels, in the plugin's order, and translateToGALabel
LABEL_BETA_ZONE = "failure-domain.beta.kubernetes.io/zone"
LABEL_BETA_REGION = "failure-domain.beta.kubernetes.io/region"
VOLUME_ZONE_LABELS = (LABEL_BETA_ZONE, LABEL_BETA_REGION, "topology.kubernetes.io/zone",
                      "topology.kubernetes.io/region")
GA_LABEL = {LABEL_BETA_ZONE: "topology.kubernetes.io/zone", LABEL_BETA_REGION: "topology.kubernetes.io/region"}
# PersistentVolume sources CSI migration translates (tryTranslatePVToCSI may
# rewrite their node affinity): refused
PV_SOURCES_MIGRATED = frozenset(("gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "azureFile", "cinder",
                                 "vsphereVolume", "portworxVolume"))


@dataclass(frozen=True)
class StorageClass:
    name: str
    provisioner: str = ""
    # volumeBindingMode after API defaulting (SetDefaults_StorageClass: Immediate)
    binding_mode: str = BINDING_IMMEDIATE
    # allowedTopologies: terms of (key, values) requirements (TopologySelectorTerm)
    allowed_topologies: Tuple[Tuple[Tuple[str, Tuple[str, ...]], ...], ...] = ()


@dataclass
class PersistentVolume:
    name: str
    labels: Dict[str, str] = field(default_factory=dict)
    storage_class: str = ""
    # spec.nodeAffinity.required.nodeSelectorTerms; None = no required affinity
    node_affinity: Optional[List[NodeSelectorTerm]] = None
    claim_ref: Optional[Tuple[str, str]] = None    # (namespace, name)
    source: str = "csi"                              # the PersistentVolumeSource field set


@dataclass
class PersistentVolumeClaim:
    name: str
    namespace: str = "default"
    volume_name: str = ""
    # storagehelpers.GetPersistentVolumeClaimClass: spec.storageClassName, else
    # the beta annotation, else ""
    storage_class: str = ""
    access_modes: Tuple[str, ...] = ()
    annotations: Dict[str, str] = field(default_factory=dict)
    deleting: bool = False

    def fully_bound(self) -> bool:
        """volumeBinder.isPVCFullyBound: a volume name and bind-completed."""
        return bool(self.volume_name) and ANN_BIND_COMPLETED in self.annotations


@dataclass
class Storage:
    pvs: Dict[str, PersistentVolume] = field(default_factory=dict)
    pvcs: Dict[Tuple[str, str], PersistentVolumeClaim] = field(default_factory=dict)   # (namespace, name)
    classes: Dict[str, StorageClass] = field(default_factory=dict)

    def claim(self, namespace: str, name: str) -> Optional[PersistentVolumeClaim]:
        return self.pvcs.get((namespace, name))

DEFAULT_BIND_ALL_HOST_IP = "0.0.0.0"


def sanitize_host_port(ip: str, protocol: str):
    """framework.HostPortInfo.sanitize: "" -> 0.0.0.0 / TCP."""
    return (ip or DEFAULT_BIND_ALL_HOST_IP), (protocol or "TCP")


@dataclass
class ImageState:
    names: Tuple[str, ...]
    size_bytes: int


@dataclass
class Node:
    name: str
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    allocatable: Dict[str, int] = field(default_factory=dict)
    unschedulable: bool = False
    images: List[ImageState] = field(default_factory=list)


# ---------------------------------------------------------------------------
# resourcehelper.PodRequests [upstream k8s.io/component-helpers/resource/helpers.go]
# ---------------------------------------------------------------------------

def _add(dst: Dict[str, int], src: Dict[str, int]):
    for k, v in src.items():
        dst[k] = dst.get(k, 0) + v


def _max(dst: Dict[str, int], src: Dict[str, int]):
    for k, v in src.items():
        if k not in dst or v > dst[k]:
            dst[k] = v


def _apply_non_missing(reqs: Dict[str, int], non_missing: Dict[str, int]) -> Dict[str, int]:
    cp = dict(reqs)
    for k, v in non_missing.items():
        if k not in reqs:
            cp[k] = cp.get(k, 0) + v
    return cp


def pod_requests(pod: Pod, non_zero: bool = False) -> Dict[str, int]:
    """Effective pod request: Σ containers, max'ed with the init-container
    high-water mark (restartable sidecars accumulate), plus overhead.  With
    `non_zero`, cpu/memory missing from a container count as 100m / 200Mi
    (the NonMissingContainerRequests option used for NonZeroRequested and for
    NodeResourcesFit scoring)."""
    nm = {CPU: DEFAULT_MILLI_CPU_REQUEST, MEMORY: DEFAULT_MEMORY_REQUEST} if non_zero else {}
    reqs: Dict[str, int] = {}
    for c in pod.containers:
        cr = _apply_non_missing(c.requests, nm) if nm else dict(c.requests)
        _add(reqs, cr)
    restartable: Dict[str, int] = {}
    init_reqs: Dict[str, int] = {}
    for c in pod.init_containers:
        cr = _apply_non_missing(c.requests, nm) if nm else dict(c.requests)
        if c.restartable:
            _add(reqs, cr)
            _add(restartable, cr)
            cr = dict(restartable)
        else:
            tmp: Dict[str, int] = {}
            _add(tmp, cr)
            _add(tmp, restartable)
            cr = tmp
        _max(init_reqs, cr)
    _max(reqs, init_reqs)
    if pod.overhead:
        _add(reqs, pod.overhead)
    return reqs


def normalized_image_name(name: str) -> str:
    """imagelocality.normalizedImageName [upstream]."""
    if name.rfind(":") <= name.rfind("/"):
        name = name + ":latest"
    return name
