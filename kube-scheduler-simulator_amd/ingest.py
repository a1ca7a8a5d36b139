"""Snapshot / record ingest into the object model.

Turns the simulator's exported cluster state into `model.Node` / `model.Pod`
and a `profile.Profile`, ready for the SoA encoder:

- `load_snapshot` reads a `ResourcesForSnap` document
  (simulator/snapshot/snapshot.go:32-41: pods, nodes, pvs, pvcs,
  storageClasses, priorityClasses, schedulerConfig, namespaces);
- `replay_records` folds a recorder file (simulator/recorder/recorder.go:39-43:
  a JSON array of {time, event Add|Update|Delete, resource}) into the final
  object set, which then loads like a snapshot;
- pods go through the simulator's apply-time mutation
  (simulator/resourceapplier/resource.go:65-81): owner references and the
  service account are dropped.  With no owner (and no Service / ReplicaSet /
  StatefulSet synced) the PodTopologySpread system-default constraints select
  nothing, so `default_spread_selector` stays None;
- pods with `spec.nodeName` are already bound (NodeInfo.AddPod at start); the
  others form the queue in PrioritySort order (priority desc, then creation
  time, then document order);
- the scheduler configuration's profile 0 becomes a `Profile`: MultiPoint
  merged onto the in-tree defaults with mergePluginSet semantics
  (simulator/scheduler/plugin/plugins.go:230-286), and the plugin args of
  NodeResourcesFit, NodeResourcesBalancedAllocation, InterPodAffinity and
  PodTopologySpread.  Settings the evaluator does not model raise
  NotImplementedError instead of being ignored.

Quantities follow k8s.io/apimachinery resource.Quantity: cpu in millicores
(`MilliValue()`), everything else in base units (`Value()`), both rounded up.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from fractions import Fraction
from math import ceil
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from . import model as m
from . import profile as P

# ---------------------------------------------------------------------------
# resource.Quantity
# ---------------------------------------------------------------------------
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_QTY = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE]|[eE][+-]?\d+)?$")


def parse_quantity(s) -> Fraction:
    """resource.ParseQuantity: sign, digits, optional fraction, one suffix
    (binary SI, decimal SI or a decimal exponent)."""
    if isinstance(s, bool):
        raise ValueError(f"quantity {s!r}")
    if isinstance(s, int):
        return Fraction(s)
    if isinstance(s, float):
        return Fraction(str(s))
    t = str(s).strip()
    mt = _QTY.match(t)
    if not mt or (not mt.group(2) and not mt.group(3)):
        raise ValueError(f"quantity {s!r}")
    sign, whole, frac, suf = mt.group(1), mt.group(2) or "0", mt.group(3) or "", mt.group(4) or ""
    v = Fraction(int(whole + frac) if (whole + frac) else 0, 10 ** len(frac))
    if suf in _BIN:
        v *= _BIN[suf]
    elif suf in _DEC:
        v *= _DEC[suf]
    else:
        v *= Fraction(10) ** int(suf[1:])
    return -v if sign == "-" else v


def milli_value(q: Fraction) -> int:
    return int(ceil(q * 1000))


def value(q: Fraction) -> int:
    return int(ceil(q))


def resource_list(d: Optional[dict]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for k, v in (d or {}).items():
        q = parse_quantity(v)
        out[k] = milli_value(q) if k == m.CPU else value(q)
    return out


# ---------------------------------------------------------------------------
# selectors
# ---------------------------------------------------------------------------
def _requirement(d: dict) -> m.Requirement:
    return m.Requirement(d["key"], d["operator"], tuple(str(x) for x in d.get("values") or ()))


def label_selector(d: Optional[dict]) -> Optional[m.LabelSelector]:
    if d is None:
        return None
    return m.LabelSelector(match_labels=tuple((k, str(v)) for k, v in (d.get("matchLabels") or {}).items()),
                           match_expressions=tuple(_requirement(r) for r in d.get("matchExpressions") or ()))


def _selector_matches(sel: m.LabelSelector, labels: Dict[str, str]) -> bool:
    """metav1.LabelSelectorAsSelector(...).Matches for namespace selectors."""
    for k, v in sel.match_labels:
        if labels.get(k) != v:
            return False
    for r in sel.match_expressions:
        has = r.key in labels
        if r.operator == m.IN:
            ok = has and labels[r.key] in r.values
        elif r.operator == m.NOT_IN:
            ok = not has or labels[r.key] not in r.values
        elif r.operator == m.EXISTS:
            ok = has
        elif r.operator == m.DOES_NOT_EXIST:
            ok = not has
        else:
            raise ValueError(f"label selector operator {r.operator!r}")
        if not ok:
            return False
    return True


def _term(d: dict) -> m.NodeSelectorTerm:
    return m.NodeSelectorTerm(match_expressions=tuple(_requirement(r) for r in d.get("matchExpressions") or ()),
                              match_fields=tuple(_requirement(r) for r in d.get("matchFields") or ()))


# A namespace no pod can have: a resolved namespaceSelector that matched nothing.
NO_NAMESPACE = "\x00none"


def _affinity_term(d: dict, ns_labels: Optional[Dict[str, Dict[str, str]]]) -> m.PodAffinityTerm:
    namespaces = tuple(d.get("namespaces") or ())
    nsel = label_selector(d.get("namespaceSelector")) if "namespaceSelector" in d else None
    if nsel is not None and not nsel.empty():
        # framework.AffinityTerm matches Namespaces ∪ {ns : selector matches its labels};
        # resolve the selector against the snapshot's namespaces.
        if ns_labels is None:
            raise NotImplementedError("namespaceSelector needs the snapshot's namespaces")
        hit = tuple(n for n in sorted(ns_labels) if _selector_matches(nsel, ns_labels[n]))
        namespaces = tuple(sorted(set(namespaces) | set(hit))) or (NO_NAMESPACE,)
        nsel = None
    return m.PodAffinityTerm(label_selector(d.get("labelSelector")), d.get("topologyKey", ""),
                             namespaces=namespaces, namespace_selector=nsel)


# ---------------------------------------------------------------------------
# objects
# ---------------------------------------------------------------------------
def node_from_k8s(obj: dict) -> m.Node:
    meta, spec, status = obj.get("metadata") or {}, obj.get("spec") or {}, obj.get("status") or {}
    taints = [m.Taint(t["key"], str(t.get("value", "")), t["effect"]) for t in spec.get("taints") or ()]
    images = [m.ImageState(tuple(i.get("names") or ()), int(i.get("sizeBytes", 0))) for i in status.get("images") or ()]
    return m.Node(name=meta["name"], labels=dict(meta.get("labels") or {}), taints=taints,
                  allocatable=resource_list(status.get("allocatable")),
                  unschedulable=bool(spec.get("unschedulable", False)), images=images)


def _container(c: dict, init: bool) -> m.Container:
    res = c.get("resources") or {}
    req = resource_list(res.get("requests"))
    # API defaulting: a request omitted next to an explicit limit defaults to the limit
    for k, v in resource_list(res.get("limits")).items():
        req.setdefault(k, v)
    ports = tuple((p.get("hostIP", ""), p.get("protocol", "TCP"), int(p["hostPort"]))
                  for p in c.get("ports") or () if p.get("hostPort"))
    return m.Container(image=c.get("image", ""), requests=req,
                       restartable=init and c.get("restartPolicy") == "Always", host_ports=ports)


def _volume(v: dict) -> Tuple[str, str, str]:
    """v1.Volume -> (name, the VolumeSource field set (its JSON key), claimName)."""
    kinds = [k for k in v if k != "name" and v[k] is not None]
    if not kinds:   # API defaulting (SetDefaults_Volume): no source set means emptyDir
        return v.get("name", ""), "emptyDir", ""
    if len(kinds) != 1:
        raise ValueError(f"volume {v.get('name')!r}: expected exactly one volume source, got {kinds}")
    kind = kinds[0]
    claim = (v[kind] or {}).get("claimName", "") if kind == "persistentVolumeClaim" else ""
    return v.get("name", ""), kind, claim


def pod_from_k8s(obj: dict, ns_labels: Optional[Dict[str, Dict[str, str]]] = None) -> m.Pod:
    """v1.Pod JSON -> model.Pod, after the simulator's mutatePods (owners and
    service account dropped: they do not enter the Filter/Score path except
    through the system-default spreading selector, which is then empty)."""
    meta, spec = obj.get("metadata") or {}, obj.get("spec") or {}
    p = m.Pod(name=meta["name"], namespace=meta.get("namespace") or "default",
              labels={k: str(v) for k, v in (meta.get("labels") or {}).items()},
              containers=[_container(c, False) for c in spec.get("containers") or ()],
              init_containers=[_container(c, True) for c in spec.get("initContainers") or ()],
              overhead=resource_list(spec["overhead"]) if spec.get("overhead") else None,
              node_name=spec.get("nodeName") or "",
              node_selector=dict(spec["nodeSelector"]) if spec.get("nodeSelector") else None,
              terminating=bool(meta.get("deletionTimestamp")))
    aff = spec.get("affinity") or {}
    na = aff.get("nodeAffinity") or {}
    req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is not None:
        p.node_affinity_required = [_term(t) for t in req.get("nodeSelectorTerms") or ()]
    pref = na.get("preferredDuringSchedulingIgnoredDuringExecution")
    if pref is not None:
        p.node_affinity_preferred = [m.PreferredSchedulingTerm(int(t["weight"]), _term(t.get("preference") or {}))
                                     for t in pref]
    for key, req_attr, pref_attr in (("podAffinity", "pod_affinity_required", "pod_affinity_preferred"),
                                     ("podAntiAffinity", "pod_anti_affinity_required",
                                      "pod_anti_affinity_preferred")):
        a = aff.get(key) or {}
        setattr(p, req_attr, [_affinity_term(t, ns_labels)
                              for t in a.get("requiredDuringSchedulingIgnoredDuringExecution") or ()])
        setattr(p, pref_attr, [m.WeightedPodAffinityTerm(int(t["weight"]), _affinity_term(t["podAffinityTerm"], ns_labels))
                               for t in a.get("preferredDuringSchedulingIgnoredDuringExecution") or ()])
    p.tolerations = [m.Toleration(t.get("key", ""), t.get("operator", ""), str(t.get("value", "")), t.get("effect", ""))
                     for t in spec.get("tolerations") or ()]
    p.volumes = [_volume(v) for v in spec.get("volumes") or ()]
    p.topology_spread_constraints = [_spread(c) for c in spec.get("topologySpreadConstraints") or ()]
    return p


def _spread(c: dict) -> m.TopologySpreadConstraint:
    """v1.TopologySpreadConstraint (a pod's, or a PodTopologySpreadArgs default)."""
    return m.TopologySpreadConstraint(int(c["maxSkew"]), c["topologyKey"], c["whenUnsatisfiable"],
                                      label_selector(c.get("labelSelector")),
                                      min_domains=int(c["minDomains"]) if c.get("minDomains") is not None else None,
                                      node_affinity_policy=c.get("nodeAffinityPolicy"),
                                      node_taints_policy=c.get("nodeTaintsPolicy"),
                                      match_label_keys=tuple(c.get("matchLabelKeys") or ()))


def _spread_json(c: m.TopologySpreadConstraint) -> dict:
    d = {"maxSkew": c.max_skew, "topologyKey": c.topology_key, "whenUnsatisfiable": c.when_unsatisfiable}
    if c.label_selector is not None:
        d["labelSelector"] = _sel_json(c.label_selector)
    if c.min_domains is not None:
        d["minDomains"] = c.min_domains
    if c.node_affinity_policy is not None:
        d["nodeAffinityPolicy"] = c.node_affinity_policy
    if c.node_taints_policy is not None:
        d["nodeTaintsPolicy"] = c.node_taints_policy
    if c.match_label_keys:
        d["matchLabelKeys"] = list(c.match_label_keys)
    return d


def pod_priority(obj: dict, classes: Dict[str, int], global_default: int) -> int:
    spec = obj.get("spec") or {}
    if spec.get("priority") is not None:
        return int(spec["priority"])
    name = spec.get("priorityClassName")
    if name:
        if name not in classes:
            raise ValueError(f"pod {obj['metadata'].get('name')}: unknown priorityClassName {name!r}")
        return classes[name]
    return global_default


def pod_preemption_policy(obj: dict, class_policy: Dict[str, str]) -> str:
    """spec.preemptionPolicy, else the one the Priority admission plugin
    copies from the pod's PriorityClass, else PreemptLowerPriority."""
    spec = obj.get("spec") or {}
    if spec.get("preemptionPolicy"):
        return spec["preemptionPolicy"]
    return class_policy.get(spec.get("priorityClassName") or "", "PreemptLowerPriority")


def rfc3339_ns(ts: Optional[str]) -> Optional[int]:
    """metav1.Time (RFC 3339, optional fraction) -> Unix nanoseconds."""
    if not ts:
        return None
    import datetime
    t = ts.strip().replace("z", "Z")
    frac = 0
    if "." in t:
        head, rest = t.split(".", 1)
        k = 0
        while k < len(rest) and rest[k].isdigit():
            k += 1
        digits, tz = rest[:k], rest[k:]
        frac = int((digits + "000000000")[:9]) if digits else 0
        t = head + tz
    dt = datetime.datetime.fromisoformat(t.replace("Z", "+00:00"))
    return int(dt.timestamp()) * 1_000_000_000 + frac


# ---------------------------------------------------------------------------
# scheduler configuration -> Profile
# ---------------------------------------------------------------------------
_POINTS_MODELLED = ("preFilter", "filter", "preScore", "score")


def _merge_plugin_set(default: List[Tuple[str, int]], custom: dict) -> List[Tuple[str, int]]:
    """mergePluginSet (plugins.go:230-286): disabled names (or "*") drop
    defaults; a re-configured default keeps its place; other custom plugins
    are appended in order."""
    disabled = {d["name"] for d in custom.get("disabled") or ()}
    enabled = [(e["name"], int(e.get("weight", 0) or 0)) for e in custom.get("enabled") or ()]
    by_name = {n: i for i, (n, _) in enumerate(enabled)}
    replaced = set()
    out: List[Tuple[str, int]] = []
    if "*" not in disabled:
        for name, w in default:
            if name in disabled:
                continue
            if name in by_name:
                i = by_name[name]
                out.append(enabled[i])
                replaced.add(i)
            else:
                out.append((name, w))
    out.extend(e for i, e in enumerate(enabled) if i not in replaced)
    return out


def profile_from_config(cfg: Optional[dict]) -> Tuple[P.Profile, Optional[int]]:
    """KubeSchedulerConfiguration (v1, JSON/YAML as a dict) -> (Profile of
    profile 0, percentageOfNodesToScore or None)."""
    prof = P.Profile()
    if not cfg:
        return prof, None
    profiles = cfg.get("profiles") or []
    if len(profiles) > 1:
        raise NotImplementedError("only profile 0 is supported (as getScorePluginWeight, plugins.go:287-289)")
    pct = cfg.get("percentageOfNodesToScore")
    if not profiles:
        return prof, pct
    p0 = profiles[0]
    plugins = p0.get("plugins") or {}
    prof.plugins = _merge_plugin_set(list(P.DEFAULT_MULTIPOINT), plugins.get("multiPoint") or {})
    # per-point sets are kept as written (ConvertForSimulator, plugins.go:177-186;
    # the in-tree MultiPoint set has nothing per point to merge with)
    for point in _POINTS_MODELLED:
        ps = plugins.get(point) or {}
        if ps.get("enabled") or ps.get("disabled"):
            prof.points[point] = ([(e["name"], int(e.get("weight", 0) or 0)) for e in ps.get("enabled") or ()],
                                  tuple(d["name"] for d in ps.get("disabled") or ()))
    prof.enabled_ids()   # refuses plugins outside the modelled in-tree set
    for f in (prof.prefilter_order, prof.filter_order, prof.prescore_order, prof.score_order):
        f()              # ... and per-point plugins the registry lacks (plugins.go:39-60)
    for pc in p0.get("pluginConfig") or ():
        name, args = pc.get("name"), pc.get("args") or {}
        if name == "NodeResourcesFit":
            ss = args.get("scoringStrategy") or {}
            t = ss.get("type", "LeastAllocated")
            if t not in P.STRATEGY_NAMES:
                raise ValueError(f"NodeResourcesFit scoringStrategy {t!r}")
            prof.fit_strategy = P.STRATEGY_NAMES[t]
            rtcr = ss.get("requestedToCapacityRatio") or {}
            prof.fit_shape = [(int(pt.get("utilization", 0)), int(pt.get("score", 0))) for pt in rtcr.get("shape") or ()]
            if ss.get("resources"):
                prof.fit_resources = [(r["name"], int(r.get("weight", 1) or 1)) for r in ss["resources"]]
            prof.fit_ignored_resources = tuple(args.get("ignoredResources") or ())
            prof.fit_ignored_resource_groups = tuple(args.get("ignoredResourceGroups") or ())
        elif name == "NodeResourcesBalancedAllocation":
            if args.get("resources"):
                prof.ba_resources = [(r["name"], int(r.get("weight", 1) or 1)) for r in args["resources"]]
        elif name == "InterPodAffinity":
            if "hardPodAffinityWeight" in args:
                prof.hard_pod_affinity_weight = int(args["hardPodAffinityWeight"])
            prof.ignore_preferred_terms_of_existing_pods = bool(args.get("ignorePreferredTermsOfExistingPods", False))
        elif name == "DefaultPreemption":
            prof.preemption_min_candidate_pct = int(args.get("minCandidateNodesPercentage", 10))
            prof.preemption_min_candidate_abs = int(args.get("minCandidateNodesAbsolute", 100))
        elif name == "PodTopologySpread":
            dt = args.get("defaultingType", "System")
            if dt not in ("System", "List"):
                raise ValueError(f"PodTopologySpread defaultingType {dt!r}")
            prof.pts_system_defaulted = dt == "System"
            prof.pts_default_constraints = [_spread(c) for c in args.get("defaultConstraints") or ()]
    prof.validate_args()   # what the scheduler's config validation refuses
    return prof, pct


# ---------------------------------------------------------------------------
# snapshot / records
# ---------------------------------------------------------------------------
@dataclass
class Snapshot:
    nodes: List[m.Node]
    pods: List[m.Pod]                       # bound pods first, then the queue in PrioritySort order
    bound: List[Tuple[int, int]]            # (pod index, node index) already running
    queue: List[int]                        # pod indices to schedule, in order
    profile: P.Profile
    skipped: List[str] = field(default_factory=list)   # pods bound to nodes absent from the snapshot


# PersistentVolumeSpec fields that are not the volume source
_PV_SPEC_FIELDS = frozenset(("capacity", "accessModes", "claimRef", "persistentVolumeReclaimPolicy",
                             "storageClassName", "mountOptions", "volumeMode", "nodeAffinity",
                             "volumeAttributesClassName"))


def storage_from_k8s(doc: dict) -> m.Storage:
    """The snapshot's pvs / pvcs / storageClasses (simulator/snapshot/
    snapshot.go:34-36) as the volume plugins' listers return them.  Classes
    get API defaulting (volumeBindingMode Immediate); a claim's or volume's
    class is the beta annotation first, then spec.storageClassName
    (storagehelpers.GetPersistentVolume[Claim]Class)."""
    st = m.Storage()
    for o in doc.get("storageClasses") or ():
        meta = o.get("metadata") or {}
        topo = tuple(tuple((e["key"], tuple(e.get("values") or ())) for e in (t.get("matchLabelExpressions") or ()))
                     for t in o.get("allowedTopologies") or ())
        st.classes[meta["name"]] = m.StorageClass(meta["name"], o.get("provisioner") or "",
                                                  o.get("volumeBindingMode") or m.BINDING_IMMEDIATE, topo)
    for o in doc.get("pvs") or ():
        meta, spec = o.get("metadata") or {}, o.get("spec") or {}
        ann = meta.get("annotations") or {}
        req = (spec.get("nodeAffinity") or {}).get("required")
        cref = spec.get("claimRef")
        srcs = [k for k in spec if k not in _PV_SPEC_FIELDS and spec[k] is not None]
        st.pvs[meta["name"]] = m.PersistentVolume(
            meta["name"], labels={k: str(v) for k, v in (meta.get("labels") or {}).items()},
            storage_class=ann.get(m.ANN_BETA_STORAGE_CLASS, spec.get("storageClassName") or ""),
            node_affinity=None if req is None else [_term(t) for t in req.get("nodeSelectorTerms") or ()],
            claim_ref=(cref.get("namespace") or "", cref.get("name") or "") if cref else None,
            source=srcs[0] if srcs else "")
    for o in doc.get("pvcs") or ():
        meta, spec = o.get("metadata") or {}, o.get("spec") or {}
        ann = dict(meta.get("annotations") or {})
        ns = meta.get("namespace") or "default"
        sc = ann[m.ANN_BETA_STORAGE_CLASS] if m.ANN_BETA_STORAGE_CLASS in ann else (spec.get("storageClassName") or "")
        st.pvcs[(ns, meta["name"])] = m.PersistentVolumeClaim(
            meta["name"], ns, volume_name=spec.get("volumeName") or "", storage_class=sc,
            access_modes=tuple(spec.get("accessModes") or ()), annotations=ann,
            deleting=bool(meta.get("deletionTimestamp")))
    return st


def load_snapshot(doc, n_nodes_check: bool = True) -> Snapshot:
    """ResourcesForSnap (dict or JSON text) -> Snapshot."""
    if isinstance(doc, (str, bytes)):
        doc = json.loads(doc)
    ns_labels = {(n.get("metadata") or {}).get("name"): dict((n.get("metadata") or {}).get("labels") or {})
                 for n in doc.get("namespaces") or ()}
    classes, global_default, class_policy = {}, 0, {}
    for pc in doc.get("priorityClasses") or ():
        classes[pc["metadata"]["name"]] = int(pc.get("value", 0))
        if pc.get("preemptionPolicy"):
            class_policy[pc["metadata"]["name"]] = pc["preemptionPolicy"]
        if pc.get("globalDefault"):
            global_default = int(pc.get("value", 0))
    nodes = [node_from_k8s(n) for n in doc.get("nodes") or ()]
    index = {n.name: i for i, n in enumerate(nodes)}
    if len(index) != len(nodes):
        raise ValueError("duplicate node names")
    bound_objs, queue_objs, skipped = [], [], []
    for k, obj in enumerate(doc.get("pods") or ()):
        node = (obj.get("spec") or {}).get("nodeName")
        if node:
            if node in index:
                bound_objs.append(obj)
            else:
                skipped.append(obj["metadata"]["name"])
        else:
            prio = pod_priority(obj, classes, global_default)
            ts = (obj.get("metadata") or {}).get("creationTimestamp") or ""
            queue_objs.append((-prio, ts, k, obj))
    queue_objs.sort(key=lambda t: t[:3])
    pods = [pod_from_k8s(o, ns_labels or None) for o in bound_objs] + \
           [pod_from_k8s(t[3], ns_labels or None) for t in queue_objs]
    storage = storage_from_k8s(doc)
    if any(p.claim_names() for p in pods):
        for n in doc.get("nodes") or ():   # NodeVolumeLimits' getVolumeLimits
            alloc = ((n.get("status") or {}).get("allocatable") or {})
            if any(k.startswith("attachable-volumes-csi-") for k in alloc):
                raise NotImplementedError(f"node {n['metadata']['name']}: CSI attach limits (NodeVolumeLimits) "
                                          "are not modelled")
    for p, o in zip(pods, bound_objs + [t[3] for t in queue_objs]):
        p.storage = storage
        p.priority = pod_priority(o, classes, global_default)
        p.preemption_policy = pod_preemption_policy(o, class_policy)
        p.start_time = rfc3339_ns((o.get("status") or {}).get("startTime"))
    bound = [(i, index[pods[i].node_name]) for i in range(len(bound_objs))]
    queue = list(range(len(bound_objs), len(pods)))
    prof, pct = profile_from_config(doc.get("schedulerConfig"))
    if n_nodes_check and pct not in (None, 100) and len(nodes) > 100:
        raise NotImplementedError(
            f"percentageOfNodesToScore={pct} with {len(nodes)} nodes: the evaluator scores every feasible node, "
            "as north_star fixes (set it to 100). Upstream's early stop (findNodesThatPassFilters stops after "
            "numFeasibleNodesToFind nodes, starting at nextStartNodeIndex) depends on which of the 16 parallel "
            "filter goroutines finishes first, so its placements are not reproducible and there is no exact "
            "result to match; at or below 100 nodes every node is scored anyway and the setting is accepted")
    for i in queue:
        pods[i].node_name = ""
    return Snapshot(nodes, pods, bound, queue, prof, skipped)


def replay_records(records) -> dict:
    """Fold recorder records (recorder.go:39-43) into a ResourcesForSnap-shaped
    document of the final objects (Add/Update replace, Delete removes)."""
    if isinstance(records, (str, bytes)):
        records = json.loads(records)
    kinds = {"Node": "nodes", "Pod": "pods", "Namespace": "namespaces", "PriorityClass": "priorityClasses",
             "PersistentVolume": "pvs", "PersistentVolumeClaim": "pvcs", "StorageClass": "storageClasses"}
    state: Dict[str, Dict[Tuple[str, str], dict]] = {v: {} for v in kinds.values()}
    order: Dict[str, List[Tuple[str, str]]] = {v: [] for v in kinds.values()}
    for r in records:
        res = r["resource"]
        kind = kinds.get(res.get("kind"))
        if kind is None:
            continue
        meta = res.get("metadata") or {}
        key = (meta.get("namespace") or "", meta["name"])
        if r["event"] == "Delete":
            state[kind].pop(key, None)
        elif r["event"] in ("Add", "Update"):
            if key not in state[kind]:
                order[kind].append(key)
            state[kind][key] = res
        else:
            raise ValueError(f"record event {r['event']!r}")
    return {kind: [state[kind][k] for k in order[kind] if k in state[kind]] for kind in kinds.values()}


# ---------------------------------------------------------------------------
# model -> k8s JSON (fixtures, round trips)
# ---------------------------------------------------------------------------
def _qty(name: str, v: int) -> str:
    return f"{v}m" if name == m.CPU else str(v)


def _sel_json(s: Optional[m.LabelSelector]):
    if s is None:
        return None
    d = {}
    if s.match_labels:
        d["matchLabels"] = dict(s.match_labels)
    if s.match_expressions:
        d["matchExpressions"] = [{"key": r.key, "operator": r.operator, "values": list(r.values)}
                                 for r in s.match_expressions]
    return d


def _term_json(t: m.NodeSelectorTerm) -> dict:
    d = {}
    if t.match_expressions:
        d["matchExpressions"] = [{"key": r.key, "operator": r.operator, "values": list(r.values)}
                                 for r in t.match_expressions]
    if t.match_fields:
        d["matchFields"] = [{"key": r.key, "operator": r.operator, "values": list(r.values)} for r in t.match_fields]
    return d


def _aff_term_json(t: m.PodAffinityTerm) -> dict:
    d = {"topologyKey": t.topology_key}
    if t.label_selector is not None:
        d["labelSelector"] = _sel_json(t.label_selector)
    if t.namespaces:
        d["namespaces"] = list(t.namespaces)
    if t.namespace_selector is not None:
        d["namespaceSelector"] = _sel_json(t.namespace_selector)
    return d


def node_to_k8s(n: m.Node) -> dict:
    spec = {}
    if n.taints:
        spec["taints"] = [{"key": t.key, "value": t.value, "effect": t.effect} for t in n.taints]
    if n.unschedulable:
        spec["unschedulable"] = True
    status = {"allocatable": {k: _qty(k, v) for k, v in n.allocatable.items()}}
    if n.images:
        status["images"] = [{"names": list(i.names), "sizeBytes": i.size_bytes} for i in n.images]
    return {"kind": "Node", "apiVersion": "v1", "metadata": {"name": n.name, "labels": dict(n.labels)},
            "spec": spec, "status": status}


def pod_to_k8s(p: m.Pod) -> dict:
    if p.default_spread_selector is not None:
        raise NotImplementedError("default_spread_selector comes from owners/services, which snapshots drop")

    def cont(c: m.Container, init: bool) -> dict:
        d = {"name": "c", "image": c.image, "resources": {"requests": {k: _qty(k, v) for k, v in c.requests.items()}}}
        if init and c.restartable:
            d["restartPolicy"] = "Always"
        if c.host_ports:
            d["ports"] = [{"hostIP": ip, "protocol": pr, "hostPort": hp, "containerPort": hp}
                          for ip, pr, hp in c.host_ports]
        return d

    spec: dict = {"containers": [cont(c, False) for c in p.containers]}
    if p.init_containers:
        spec["initContainers"] = [cont(c, True) for c in p.init_containers]
    if p.overhead:
        spec["overhead"] = {k: _qty(k, v) for k, v in p.overhead.items()}
    if p.node_name:
        spec["nodeName"] = p.node_name
    if p.node_selector is not None:
        spec["nodeSelector"] = dict(p.node_selector)
    aff: dict = {}
    na: dict = {}
    if p.node_affinity_required is not None:
        na["requiredDuringSchedulingIgnoredDuringExecution"] = {
            "nodeSelectorTerms": [_term_json(t) for t in p.node_affinity_required]}
    if p.node_affinity_preferred is not None:
        na["preferredDuringSchedulingIgnoredDuringExecution"] = [
            {"weight": t.weight, "preference": _term_json(t.preference)} for t in p.node_affinity_preferred]
    if na:
        aff["nodeAffinity"] = na
    for key, req, pref in (("podAffinity", p.pod_affinity_required, p.pod_affinity_preferred),
                           ("podAntiAffinity", p.pod_anti_affinity_required, p.pod_anti_affinity_preferred)):
        d = {}
        if req:
            d["requiredDuringSchedulingIgnoredDuringExecution"] = [_aff_term_json(t) for t in req]
        if pref:
            d["preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": w.weight, "podAffinityTerm": _aff_term_json(w.term)} for w in pref]
        if d:
            aff[key] = d
    if aff:
        spec["affinity"] = aff
    if p.tolerations:
        spec["tolerations"] = [{k: v for k, v in (("key", t.key), ("operator", t.operator), ("value", t.value),
                                                  ("effect", t.effect)) if v} for t in p.tolerations]
    if p.topology_spread_constraints:
        spec["topologySpreadConstraints"] = [_spread_json(c) for c in p.topology_spread_constraints]
    if p.priority:
        spec["priority"] = p.priority
    if p.preemption_policy != "PreemptLowerPriority":
        spec["preemptionPolicy"] = p.preemption_policy
    meta = {"name": p.name, "namespace": p.namespace, "labels": dict(p.labels)}
    if p.terminating:
        meta["deletionTimestamp"] = "2024-01-01T00:00:00Z"
    out = {"kind": "Pod", "apiVersion": "v1", "metadata": meta, "spec": spec}
    if p.start_time is not None:
        out["status"] = {"startTime": ns_rfc3339(p.start_time)}
    return out


def ns_rfc3339(ns: int) -> str:
    import datetime
    sec, frac = divmod(int(ns), 1_000_000_000)
    t = datetime.datetime.fromtimestamp(sec, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S")
    return t + (f".{frac:09d}".rstrip("0") if frac else "") + "Z"


def profile_to_config(prof: P.Profile) -> dict:
    """Profile -> KubeSchedulerConfiguration with an explicit multiPoint list."""
    inv = {v: k for k, v in P.STRATEGY_NAMES.items()}
    pcs = [
        {"name": "NodeResourcesFit", "args": {"scoringStrategy": {
            "type": inv[prof.fit_strategy], "resources": [{"name": n, "weight": w} for n, w in prof.fit_resources]},
            "ignoredResources": list(prof.fit_ignored_resources),
            "ignoredResourceGroups": list(prof.fit_ignored_resource_groups)}},
        {"name": "NodeResourcesBalancedAllocation",
         "args": {"resources": [{"name": n, "weight": w} for n, w in prof.ba_resources]}},
        {"name": "InterPodAffinity", "args": {"hardPodAffinityWeight": prof.hard_pod_affinity_weight,
                                              "ignorePreferredTermsOfExistingPods":
                                                  prof.ignore_preferred_terms_of_existing_pods}},
        {"name": "PodTopologySpread", "args": {"defaultingType": "System" if prof.pts_system_defaulted else "List",
                                               "defaultConstraints": [_spread_json(c)
                                                                      for c in prof.pts_default_constraints]}},
    ]
    if prof.fit_strategy == P.REQUESTED_TO_CAPACITY_RATIO:
        pcs[0]["args"]["scoringStrategy"]["requestedToCapacityRatio"] = {
            "shape": [{"utilization": u, "score": sc} for u, sc in prof.fit_shape]}
    return {"apiVersion": "kubescheduler.config.k8s.io/v1", "kind": "KubeSchedulerConfiguration",
            "percentageOfNodesToScore": 100,
            "profiles": [{"schedulerName": "default-scheduler",
                          "plugins": {"multiPoint": {"enabled": [{"name": n, "weight": w} for n, w in prof.plugins],
                                                     "disabled": [{"name": "*"}]}},
                          "pluginConfig": pcs}]}


def snapshot_document(nodes: Sequence[m.Node], pods: Sequence[m.Pod], prof: P.Profile,
                      namespaces: Iterable[Tuple[str, Dict[str, str]]] = ()) -> dict:
    """A ResourcesForSnap document for (nodes, pods, profile)."""
    return {"pods": [pod_to_k8s(p) for p in pods], "nodes": [node_to_k8s(n) for n in nodes], "pvs": [],
            "pvcs": [], "storageClasses": [], "priorityClasses": [], "schedulerConfig": profile_to_config(prof),
            "namespaces": [{"metadata": {"name": n, "labels": dict(lb)}} for n, lb in namespaces]}
