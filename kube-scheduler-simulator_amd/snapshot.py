"""ctypes binding of the native snapshot encoder (include/ksched_snapshot.h).

`Snapshot` hands the cluster objects (model.py: the subset of v1.Node /
v1.Pod / NodeInfo the in-tree plugins read) to libksched.so as the flat C
views a cgo caller would build from the real objects, and the library encodes
them (the C++ restatement in csrc/ksched_snapshot.cpp).  The views are only
alive for the duration of each call, as under the cgo pointer rules.

`Snapshot.load(engine)` / `sync(engine)` put the encoding onto a device
context; `status()` / `prefilter()` give the framework.Status codes and
messages the Go shim returns from Filter / PreFilter.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import encoder as E
from . import model as m
from . import native
from . import profile as P

cp = C.c_char_p
i32 = C.c_int32
i64 = C.c_int64


def _b(s: Optional[str]) -> Optional[bytes]:
    return None if s is None else s.encode("utf-8", errors="surrogatepass")


class StrPair(C.Structure):
    _fields_ = [("key", cp), ("value", cp)]


class Quantity(C.Structure):
    _fields_ = [("name", cp), ("value", i64)]


class TaintView(C.Structure):
    _fields_ = [("key", cp), ("value", cp), ("effect", cp)]


class TolerationView(C.Structure):
    _fields_ = [("key", cp), ("op", cp), ("value", cp), ("effect", cp)]


class RequirementView(C.Structure):
    _fields_ = [("key", cp), ("op", cp), ("n_values", i32), ("values", C.POINTER(cp))]


class NodeSelectorTermView(C.Structure):
    _fields_ = [("n_expr", i32), ("expr", C.POINTER(RequirementView)), ("n_fields", i32),
                ("fields", C.POINTER(RequirementView))]


class PreferredTermView(C.Structure):
    _fields_ = [("weight", i32), ("preference", NodeSelectorTermView)]


class LabelSelectorView(C.Structure):
    _fields_ = [("is_set", i32), ("n_labels", i32), ("match_labels", C.POINTER(StrPair)), ("n_expr", i32),
                ("expr", C.POINTER(RequirementView))]


class AffinityTermView(C.Structure):
    _fields_ = [("weight", i32), ("selector", LabelSelectorView), ("topology_key", cp), ("n_namespaces", i32),
                ("namespaces", C.POINTER(cp)), ("namespace_selector", LabelSelectorView)]


class SpreadView(C.Structure):
    _fields_ = [("max_skew", i32), ("topology_key", cp), ("when_unsatisfiable", cp), ("selector", LabelSelectorView),
                ("min_domains", i32), ("node_affinity_policy", cp), ("node_taints_policy", cp),
                ("n_match_label_keys", i32), ("match_label_keys", C.POINTER(cp))]


class HostPortView(C.Structure):
    _fields_ = [("host_ip", cp), ("protocol", cp), ("host_port", i32), ("pad", i32)]


class ContainerView(C.Structure):
    _fields_ = [("image", cp), ("n_requests", i32), ("requests", C.POINTER(Quantity)), ("restartable", i32),
                ("n_host_ports", i32), ("host_ports", C.POINTER(HostPortView))]


class ImageView(C.Structure):
    _fields_ = [("n_names", i32), ("names", C.POINTER(cp)), ("size_bytes", i64)]


class NodeView(C.Structure):
    _fields_ = [("name", cp), ("n_labels", i32), ("labels", C.POINTER(StrPair)), ("n_taints", i32),
                ("taints", C.POINTER(TaintView)), ("n_alloc", i32), ("allocatable", C.POINTER(Quantity)),
                ("unschedulable", i32), ("n_images", i32), ("images", C.POINTER(ImageView))]


class VolumeView(C.Structure):
    _fields_ = [("name", cp), ("kind", cp), ("claim_name", cp)]


class PVView(C.Structure):
    _fields_ = [("name", cp), ("n_labels", i32), ("labels", C.POINTER(StrPair)), ("storage_class", cp),
                ("claim_namespace", cp), ("claim_name", cp), ("source", cp), ("has_node_affinity", i32),
                ("n_terms", i32), ("terms", C.POINTER(NodeSelectorTermView))]


class PVCView(C.Structure):
    _fields_ = [("namespace_", cp), ("name", cp), ("volume_name", cp), ("storage_class", cp),
                ("n_access_modes", i32), ("access_modes", C.POINTER(cp)), ("n_annotations", i32),
                ("annotations", C.POINTER(StrPair)), ("deleting", i32)]


class TopologyRequirementView(C.Structure):
    _fields_ = [("key", cp), ("n_values", i32), ("values", C.POINTER(cp))]


class TopologyTermView(C.Structure):
    _fields_ = [("n_requirements", i32), ("requirements", C.POINTER(TopologyRequirementView))]


class StorageClassView(C.Structure):
    _fields_ = [("name", cp), ("provisioner", cp), ("binding_mode", cp), ("n_allowed_topologies", i32),
                ("allowed_topologies", C.POINTER(TopologyTermView))]


class PodView(C.Structure):
    _fields_ = [
        ("namespace_", cp), ("name", cp), ("n_labels", i32), ("labels", C.POINTER(StrPair)),
        ("n_containers", i32), ("containers", C.POINTER(ContainerView)),
        ("n_init_containers", i32), ("init_containers", C.POINTER(ContainerView)),
        ("has_overhead", i32), ("n_overhead", i32), ("overhead", C.POINTER(Quantity)),
        ("node_name", cp),
        ("has_node_selector", i32), ("n_node_selector", i32), ("node_selector", C.POINTER(StrPair)),
        ("has_na_required", i32), ("n_na_required", i32), ("na_required", C.POINTER(NodeSelectorTermView)),
        ("has_na_preferred", i32), ("n_na_preferred", i32), ("na_preferred", C.POINTER(PreferredTermView)),
        ("n_pod_affinity_required", i32), ("pod_affinity_required", C.POINTER(AffinityTermView)),
        ("n_pod_affinity_preferred", i32), ("pod_affinity_preferred", C.POINTER(AffinityTermView)),
        ("n_pod_anti_affinity_required", i32), ("pod_anti_affinity_required", C.POINTER(AffinityTermView)),
        ("n_pod_anti_affinity_preferred", i32), ("pod_anti_affinity_preferred", C.POINTER(AffinityTermView)),
        ("n_tolerations", i32), ("tolerations", C.POINTER(TolerationView)),
        ("n_spread", i32), ("spread", C.POINTER(SpreadView)),
        ("default_spread_selector", LabelSelectorView),
        ("terminating", i32), ("priority", i32), ("n_volumes", i32), ("volumes", C.POINTER(VolumeView))]


class PluginView(C.Structure):
    _fields_ = [("name", cp), ("weight", i32)]


class PluginSetView(C.Structure):
    _fields_ = [("n_enabled", i32), ("enabled", C.POINTER(PluginView)), ("n_disabled", i32),
                ("disabled", C.POINTER(cp))]


# ksg_profile_view.points index (KSG_POINT_*) of profile.Profile.points keys
POINTS = ("preFilter", "filter", "preScore", "score")
NPOINTS = len(POINTS)


class ProfileView(C.Structure):
    _fields_ = [("n_plugins", i32), ("plugins", C.POINTER(PluginView)), ("fit_strategy", cp),
                ("n_fit_resources", i32), ("fit_resources", C.POINTER(Quantity)),
                ("n_ba_resources", i32), ("ba_resources", C.POINTER(Quantity)),
                ("n_fit_ignored_resources", i32), ("fit_ignored_resources", C.POINTER(cp)),
                ("n_fit_ignored_groups", i32), ("fit_ignored_groups", C.POINTER(cp)),
                ("hard_pod_affinity_weight", i32), ("ignore_preferred_terms_of_existing_pods", i32),
                ("pts_system_defaulted", i32), ("ba_skip_best_effort", i32),
                ("points", PluginSetView * NPOINTS), ("n_shape", i32), ("shape_utilization", C.POINTER(i32)),
                ("shape_score", C.POINTER(i32)), ("n_default_constraints", i32),
                ("default_constraints", C.POINTER(SpreadView))]


class ProfileInfo(C.Structure):
    """ksg_profile_info: per-point run orders and the two weight maps."""
    _fields_ = [("n_order", i32 * NPOINTS), ("order", (i32 * native.NPLUGINS) * NPOINTS),
                ("store_weight", i64 * native.NPLUGINS), ("selection_weight", i32 * native.NPLUGINS),
                ("normalize_mask", C.c_uint32), ("pad", i32)]


class _Keep:
    """Builds C arrays and keeps every buffer alive until the call returns."""

    def __init__(self):
        self.refs = []

    def arr(self, ctype, items):
        a = (ctype * max(len(items), 1))(*items)
        self.refs.append(a)
        return len(items), a

    def strs(self, items):
        return self.arr(cp, [_b(s) for s in items])

    def pairs(self, d):
        return self.arr(StrPair, [StrPair(_b(k), _b(v)) for k, v in d.items()])

    def res(self, d):
        return self.arr(Quantity, [Quantity(_b(k), int(v)) for k, v in d.items()])

    def reqs(self, rs):
        out = []
        for r in rs:
            n, vals = self.strs(list(r.values))
            out.append(RequirementView(_b(r.key), _b(r.operator), n, vals))
        return self.arr(RequirementView, out)

    def term(self, t: m.NodeSelectorTerm):
        ne, e = self.reqs(t.match_expressions)
        nf, f = self.reqs(t.match_fields)
        return NodeSelectorTermView(ne, e, nf, f)

    def sel(self, ls: Optional[m.LabelSelector]):
        if ls is None:
            return LabelSelectorView()
        nl, lab = self.arr(StrPair, [StrPair(_b(k), _b(v)) for k, v in ls.match_labels])
        ne, e = self.reqs(ls.match_expressions)
        return LabelSelectorView(1, nl, lab, ne, e)

    def aff(self, terms, weighted: bool):
        out = []
        for x in terms:
            w, t = (x.weight, x.term) if weighted else (0, x)
            nn, ns = self.strs(list(t.namespaces))
            out.append(AffinityTermView(w, self.sel(t.label_selector), _b(t.topology_key), nn, ns,
                                        self.sel(t.namespace_selector)))
        return self.arr(AffinityTermView, out)

    def containers(self, cs):
        out = []
        for c in cs:
            n, rq = self.res(c.requests)
            nh, hp = self.arr(HostPortView, [HostPortView(_b(ip), _b(proto), int(port), 0)
                                             for ip, proto, port in c.host_ports])
            out.append(ContainerView(_b(c.image), n, rq, 1 if c.restartable else 0, nh, hp))
        return self.arr(ContainerView, out)


def node_view(n: m.Node, k: _Keep) -> NodeView:
    nl, lab = k.pairs(n.labels)
    nt, ts = k.arr(TaintView, [TaintView(_b(t.key), _b(t.value), _b(t.effect)) for t in n.taints])
    na, al = k.res(n.allocatable)
    imgs = []
    for im in n.images:
        nn, names = k.strs(list(im.names))
        imgs.append(ImageView(nn, names, int(im.size_bytes)))
    ni, iv = k.arr(ImageView, imgs)
    return NodeView(_b(n.name), nl, lab, nt, ts, na, al, 1 if n.unschedulable else 0, ni, iv)


def pod_view(p: m.Pod, k: _Keep) -> PodView:
    v = PodView()
    v.namespace_, v.name = _b(p.namespace), _b(p.name)
    v.n_labels, v.labels = k.pairs(p.labels)
    v.n_containers, v.containers = k.containers(p.containers)
    v.n_init_containers, v.init_containers = k.containers(p.init_containers)
    if p.overhead is not None:
        v.has_overhead = 1
        v.n_overhead, v.overhead = k.res(p.overhead)
    v.node_name = _b(p.node_name or "")
    if p.node_selector is not None:
        v.has_node_selector = 1
        v.n_node_selector, v.node_selector = k.pairs(p.node_selector)
    if p.node_affinity_required is not None:
        v.has_na_required = 1
        v.n_na_required, v.na_required = k.arr(NodeSelectorTermView, [k.term(t) for t in p.node_affinity_required])
    if p.node_affinity_preferred is not None:
        v.has_na_preferred = 1
        v.n_na_preferred, v.na_preferred = k.arr(
            PreferredTermView, [PreferredTermView(t.weight, k.term(t.preference)) for t in p.node_affinity_preferred])
    v.n_pod_affinity_required, v.pod_affinity_required = k.aff(p.pod_affinity_required, False)
    v.n_pod_affinity_preferred, v.pod_affinity_preferred = k.aff(p.pod_affinity_preferred, True)
    v.n_pod_anti_affinity_required, v.pod_anti_affinity_required = k.aff(p.pod_anti_affinity_required, False)
    v.n_pod_anti_affinity_preferred, v.pod_anti_affinity_preferred = k.aff(p.pod_anti_affinity_preferred, True)
    v.n_tolerations, v.tolerations = k.arr(
        TolerationView, [TolerationView(_b(t.key), _b(t.operator), _b(t.value), _b(t.effect)) for t in p.tolerations])
    v.n_spread, v.spread = k.arr(SpreadView, [_spread_view(c, k) for c in p.topology_spread_constraints])
    v.default_spread_selector = k.sel(p.default_spread_selector)
    v.terminating = 1 if p.terminating else 0
    v.priority = int(p.priority)
    v.n_volumes, v.volumes = k.arr(VolumeView, [VolumeView(_b(n), _b(kind), _b(claim)) for n, kind, claim in p.volumes])
    return v


def pv_view(pv: m.PersistentVolume, k: _Keep) -> PVView:
    n, labels = k.pairs(pv.labels)
    v = PVView(_b(pv.name), n, labels, _b(pv.storage_class or ""))
    if pv.claim_ref is not None:
        v.claim_namespace, v.claim_name = _b(pv.claim_ref[0]), _b(pv.claim_ref[1])
    v.source = _b(pv.source or "")
    if pv.node_affinity is not None:
        v.has_node_affinity = 1
        v.n_terms, v.terms = k.arr(NodeSelectorTermView, [k.term(t) for t in pv.node_affinity])
    return v


def pvc_view(c: m.PersistentVolumeClaim, k: _Keep) -> PVCView:
    nm, modes = k.strs(list(c.access_modes))
    na, ann = k.pairs(c.annotations)
    return PVCView(_b(c.namespace), _b(c.name), _b(c.volume_name or ""), _b(c.storage_class or ""), nm, modes,
                   na, ann, 1 if c.deleting else 0)


def storage_class_view(sc: m.StorageClass, k: _Keep) -> StorageClassView:
    terms = []
    for term in sc.allowed_topologies:
        reqs = []
        for key, vals in term:
            nv, vs = k.strs(list(vals))
            reqs.append(TopologyRequirementView(_b(key), nv, vs))
        nr, ra = k.arr(TopologyRequirementView, reqs)
        terms.append(TopologyTermView(nr, ra))
    nt, ta = k.arr(TopologyTermView, terms)
    return StorageClassView(_b(sc.name), _b(sc.provisioner or ""), _b(sc.binding_mode or ""), nt, ta)


def _spread_view(c: m.TopologySpreadConstraint, k: _Keep) -> SpreadView:
    nk, keys = k.strs(list(c.match_label_keys))
    return SpreadView(c.max_skew, _b(c.topology_key), _b(c.when_unsatisfiable), k.sel(c.label_selector),
                      c.min_domains if c.min_domains is not None else 0,
                      _b(c.node_affinity_policy or ""), _b(c.node_taints_policy or ""), nk, keys)


def profile_view(prof: P.Profile, k: _Keep) -> ProfileView:
    n, pl = k.arr(PluginView, [PluginView(_b(nm), int(w)) for nm, w in prof.plugins])
    nf, fr = k.arr(Quantity, [Quantity(_b(r), int(w)) for r, w in prof.fit_resources])
    nb, br = k.arr(Quantity, [Quantity(_b(r), int(w)) for r, w in prof.ba_resources])
    ni, ig = k.strs(list(prof.fit_ignored_resources))
    ng, gr = k.strs(list(prof.fit_ignored_resource_groups))
    strat = {v: n for n, v in P.STRATEGY_NAMES.items()}[prof.fit_strategy]
    v = ProfileView(n, pl, _b(strat), nf, fr, nb, br, ni, ig, ng, gr, int(prof.hard_pod_affinity_weight),
                    1 if prof.ignore_preferred_terms_of_existing_pods else 0,
                    1 if prof.pts_system_defaulted else 0, 1 if prof.ba_skip_best_effort else 0)
    for idx, point in enumerate(POINTS):
        if point not in prof.points:
            continue
        enabled, disabled = prof.points[point]
        ne, en = k.arr(PluginView, [PluginView(_b(nm), int(w)) for nm, w in enabled])
        nd, dis = k.strs(list(disabled))
        v.points[idx] = PluginSetView(ne, en, nd, dis)
    v.n_shape, v.shape_utilization = k.arr(i32, [int(u) for u, _ in prof.fit_shape])
    _, v.shape_score = k.arr(i32, [int(sc) for _, sc in prof.fit_shape])
    v.n_default_constraints, v.default_constraints = k.arr(
        SpreadView, [_spread_view(c, k) for c in prof.pts_default_constraints])
    return v


CODE_SUCCESS, CODE_UNSCHEDULABLE, CODE_UNRESOLVABLE, CODE_SKIP = 0, 2, 3, 5   # framework.Code


class SnapshotError(RuntimeError):
    pass


class Snapshot:
    """ksg_snapshot: the native encoder over the cluster objects."""

    def __init__(self, prof: P.Profile, nodes: Sequence[m.Node] = (), pods: Sequence[m.Pod] = (),
                 bound: Sequence[Tuple[int, int]] = (), lib_path: Optional[str] = None,
                 namespaces: Sequence[Tuple[str, Dict[str, str]]] = ()):
        import os
        path = lib_path or native.LIB_PATH
        if not os.path.exists(path):
            raise native.KschedError(f"{path} not found: run __graft_entry__.build()")
        self.lib = C.CDLL(path)
        f = native._bind(self.lib, "ksg_snapshot_")
        vp = C.c_void_p
        self._new = f("new", C.c_int, C.POINTER(ProfileView), C.POINTER(vp))
        self._free = f("free", C.c_int, vp)
        self._err = f("error", cp, vp)
        self._add_node = f("add_node", C.c_int, vp, C.POINTER(NodeView), C.POINTER(i32))
        self._add_pod = f("add_pod", C.c_int, vp, C.POINTER(PodView), C.POINTER(i32))
        self._add_ns = f("add_namespace", C.c_int, vp, cp, i32, C.POINTER(StrPair))
        self._add_pv = f("add_pv", C.c_int, vp, C.POINTER(PVView))
        self._add_pvc = f("add_pvc", C.c_int, vp, C.POINTER(PVCView))
        self._add_sc = f("add_storage_class", C.c_int, vp, C.POINTER(StorageClassView))
        self._prefilter_msg = f("prefilter_message", C.c_int, vp, i32, i32, C.c_char_p, i32, C.POINTER(i32))
        self._hint_pod = f("hint_pod", C.c_int, vp, C.POINTER(PodView))
        self._unhint_pod = f("unhint_pod", C.c_int, vp, cp, cp)
        self._bind_ = f("bind", C.c_int, vp, i32, i32)
        self._encode = f("encode", C.c_int, vp)
        self._encode_inc = f("encode_incremental", C.c_int, vp, C.POINTER(i32))
        self._view = f("view", C.c_int, vp, C.POINTER(native.KsgNodes), C.POINTER(native.KsgTopology),
                       C.POINTER(native.KsgWorkload), C.POINTER(native.KsgProfile))
        self._load = f("load", C.c_int, vp, vp)
        self._sync = f("sync", C.c_int, vp, vp, C.POINTER(i32))
        self._assume = f("assume", C.c_int, vp, vp, i32, i32)
        self._forget = f("forget", C.c_int, vp, vp, i32, i32)
        self._status = f("status", C.c_int, vp, i32, C.c_uint32, i32, C.POINTER(i32), C.c_char_p, i32,
                         C.POINTER(i32))
        self._prefilter = f("prefilter", C.c_int, vp, i32, i32, C.c_uint32, C.POINTER(i32), C.POINTER(i32),
                            C.POINTER(cp), i32, C.POINTER(i32))
        self._profile_info = f("profile_info", C.c_int, vp, C.POINTER(ProfileInfo))
        self._statuses = f("statuses", C.c_int, vp, i32, C.POINTER(C.c_uint32), i32, C.POINTER(i32),
                           C.POINTER(i32), C.c_char_p, i64, C.POINTER(i32), C.POINTER(i64))
        self._statuses_kept = f("statuses_kept", C.c_int, vp, i32, C.POINTER(C.c_uint32), i32,
                                C.POINTER(C.POINTER(i32)), C.POINTER(C.POINTER(i32)), C.c_char_p, i64,
                                C.POINTER(i32), C.POINTER(i64))
        self._kept_stats = f("statuses_kept_stats", C.c_int, vp, C.POINTER(i64), C.POINTER(i64))
        self._clear_storage = f("clear_storage", C.c_int, vp)
        self.h = vp()
        k = _Keep()
        rc = self._new(C.byref(profile_view(prof, k)), C.byref(self.h))
        if rc != 0:
            raise SnapshotError(f"ksg_snapshot_new rc={rc}")
        native.track(self)
        self.prof = prof
        self.n_pods = 0
        for name, labels in namespaces:
            self.add_namespace(name, labels)
        for n in nodes:
            self.add_node(n)
        # the volume plugins' listers: the storage objects the pods' claims
        # resolve against (model.Pod.storage; one Storage shared by the pods)
        for st in {id(p.storage): p.storage for p in pods if p.storage is not None}.values():
            self.add_storage(st)
        for p in pods:
            self.add_pod(p)
        for pi, ni in bound:
            self.bind(pi, ni)

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise SnapshotError(f"ksg_snapshot_{what} rc={rc}: {self._err(self.h).decode()}")

    def close(self):
        if self.h:
            self._free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- building ---------------------------------------------------------
    def add_node(self, n: m.Node) -> int:
        k = _Keep()
        idx = i32()
        self._check(self._add_node(self.h, C.byref(node_view(n, k)), C.byref(idx)), "add_node")
        return idx.value

    def add_namespace(self, name: str, labels: Dict[str, str]) -> None:
        k = _Keep()
        n, arr = k.pairs(labels)
        self._check(self._add_ns(self.h, _b(name), n, arr), "add_namespace")

    def add_storage(self, st: m.Storage) -> None:
        """ksg_snapshot_add_pv / _add_pvc / _add_storage_class of every object."""
        for sc in st.classes.values():
            k = _Keep()
            self._check(self._add_sc(self.h, C.byref(storage_class_view(sc, k))), "add_storage_class")
        for pv in st.pvs.values():
            k = _Keep()
            self._check(self._add_pv(self.h, C.byref(pv_view(pv, k))), "add_pv")
        for c in st.pvcs.values():
            k = _Keep()
            self._check(self._add_pvc(self.h, C.byref(pvc_view(c, k))), "add_pvc")

    def clear_storage(self) -> None:
        """ksg_snapshot_clear_storage: drop every PV, claim and StorageClass
        (a lister resync: clear, then add_storage of what is left)."""
        self._check(self._clear_storage(self.h), "clear_storage")

    def prefilter_message(self, pod: int, plugin: int) -> str:
        """ksg_snapshot_prefilter_message: the plugin's PreFilter rejection ("" none)."""
        n = i32()
        self._check(self._prefilter_msg(self.h, pod, plugin, None, 0, C.byref(n)), "prefilter_message")
        buf = C.create_string_buffer(n.value + 1)
        self._check(self._prefilter_msg(self.h, pod, plugin, buf, n.value + 1, C.byref(n)), "prefilter_message")
        return buf.value.decode()

    def add_pod(self, p: m.Pod) -> int:
        k = _Keep()
        idx = i32()
        self._check(self._add_pod(self.h, C.byref(pod_view(p, k)), C.byref(idx)), "add_pod")
        self.n_pods = idx.value + 1
        return idx.value

    def add_pod_view(self, view: "PodView") -> int:
        """ksg_snapshot_add_pod of a view built beforehand (pod_view; its
        buffers kept alive by the caller): the per-cycle call alone."""
        idx = i32()
        self._check(self._add_pod(self.h, C.byref(view), C.byref(idx)), "add_pod")
        self.n_pods = idx.value + 1
        return idx.value

    def hint_pod(self, p: m.Pod) -> None:
        """ksg_snapshot_hint_pod: a pending pod's selectors / templates join the
        encoding universe now, so its later add_pod appends in place."""
        k = _Keep()
        self._check(self._hint_pod(self.h, C.byref(pod_view(p, k))), "hint_pod")

    def unhint_pod(self, namespace: str, name: str) -> None:
        """ksg_snapshot_unhint_pod: a hinted pending pod was deleted."""
        self._check(self._unhint_pod(self.h, _b(namespace), _b(name)), "unhint_pod")

    def bind(self, pod: int, node: int):
        self._check(self._bind_(self.h, pod, node), "bind")

    # -- encoding ---------------------------------------------------------
    def encode(self):
        self._check(self._encode(self.h), "encode")

    def encode_incremental(self) -> bool:
        """Encode the pods added since the last encode; True when they were
        appended to the loaded universe, False after a full re-encode."""
        ap = i32()
        self._check(self._encode_inc(self.h, C.byref(ap)), "encode_incremental")
        return bool(ap.value)

    def arrays(self) -> dict:
        """The encoded SoA as numpy copies (same names as encoder.py's)."""
        nd, tp, wl, pf = native.KsgNodes(), native.KsgTopology(), native.KsgWorkload(), native.KsgProfile()
        self._check(self._view(self.h, C.byref(nd), C.byref(tp), C.byref(wl), C.byref(pf)), "view")
        N, R, L = nd.n_nodes, nd.n_res, max(nd.n_label_cols, 1)

        def a(ptr, count, dtype, shape=None):
            out = np.ctypeslib.as_array(ptr, shape=(count,)).astype(dtype, copy=True)
            return out.reshape(shape) if shape else out
        T = max(tp.n_templates, 1)
        out = {
            "alloc": a(nd.alloc, R * N, np.int64, (R, N)),
            "requested": a(nd.requested, R * N, np.int64, (R, N)),
            "nonzero": a(nd.nonzero, 2 * N, np.int64, (2, N)),
            "allowed_pods": a(nd.allowed_pods, N, np.int32),
            "pod_count": a(nd.pod_count, N, np.int32),
            "unschedulable": a(nd.unschedulable, N, np.uint8),
            "label_val": a(nd.label_val, L * N, np.uint32, (L, N)),
            "label_num": a(nd.label_num, L * N, np.int64, (L, N)),
            "label_num_ok": a(nd.label_num_ok, L * N, np.uint8, (L, N)),
            "taints": a(nd.taints, nd.max_taints * N, np.uint32, (nd.max_taints, N)),
            "taint_effect": a(nd.taint_effect, max(nd.n_taint_vocab, 1), np.uint8),
            "images": a(nd.images, nd.max_images * N, np.uint32, (nd.max_images, N)),
            "col_vocab": a(tp.col_vocab, L, np.int32),
            "col_unique": a(tp.col_unique, L, np.uint8),
            "tmpl_col": a(tp.tmpl_col, T, np.int32),
            "tmpl_kind": a(tp.tmpl_kind, T, np.int32),
            "tmpl_weight": a(tp.tmpl_weight, T, np.int32),
            "log_table": a(tp.log_table, tp.log_n, np.float64),
            "pods": np.frombuffer(C.string_at(wl.pods, wl.n_pods * E.POD_DTYPE.itemsize),
                                  dtype=E.POD_DTYPE).copy(),
            "prog": a(wl.prog, wl.prog_len, np.int32),
        }
        out["profile"] = {f: (list(getattr(pf, f)) if isinstance(getattr(pf, f), C.Array) else getattr(pf, f))
                          for f, _ in native.KsgProfile._fields_}
        out["meta"] = {"n_label_cols": nd.n_label_cols, "n_taint_vocab": nd.n_taint_vocab, "n_images": nd.n_images,
                       "n_port_vocab": nd.n_port_vocab,
                       "n_selectors": tp.n_selectors, "n_templates": tp.n_templates, "n_res": R}
        return out

    # -- device -----------------------------------------------------------
    def load(self, engine: native.Engine):
        self._check(self._load(self.h, engine.ctx), "load")
        engine._snapshot_loaded(self)

    def sync(self, engine: native.Engine) -> bool:
        """True when the new pods were appended, False after a full reload."""
        ap = i32()
        self._check(self._sync(self.h, engine.ctx, C.byref(ap)), "sync")
        engine._snapshot_loaded(self)
        return bool(ap.value)

    def assume(self, engine: native.Engine, pod: int, node: int):
        self._check(self._assume(self.h, engine.ctx, pod, node), "assume")

    def forget(self, engine: native.Engine, pod: int, node: int):
        self._check(self._forget(self.h, engine.ctx, pod, node), "forget")

    def profile_info(self) -> dict:
        """ksg_snapshot_profile_info: {point: [plugin ids]}, store / selection
        weights by plugin name (0 entries dropped), normalize mask."""
        pi = ProfileInfo()
        self._check(self._profile_info(self.h, C.byref(pi)), "profile_info")
        out = {pt: [pi.order[k][i] for i in range(pi.n_order[k])] for k, pt in enumerate(POINTS)}
        out["store_weight"] = {P.PLUGIN_NAMES[i]: int(pi.store_weight[i]) for i in range(native.NPLUGINS)
                               if pi.store_weight[i]}
        out["selection_weight"] = {P.PLUGIN_NAMES[i]: int(pi.selection_weight[i]) for i in range(native.NPLUGINS)
                                   if pi.selection_weight[i]}
        out["normalize_mask"] = int(pi.normalize_mask)
        return out

    # -- framework.Status --------------------------------------------------
    def status(self, pod: int, word: int, node: int) -> Tuple[int, str]:
        code, ln = i32(), i32()
        buf = C.create_string_buffer(512)
        self._check(self._status(self.h, pod, word, node, C.byref(code), buf, 512, C.byref(ln)), "status")
        if ln.value >= 512:
            buf = C.create_string_buffer(ln.value + 1)
            self._check(self._status(self.h, pod, word, node, C.byref(code), buf, ln.value + 1, C.byref(ln)),
                        "status")
        return code.value, buf.value.decode("utf-8")

    def statuses(self, pod: int, words) -> Tuple[np.ndarray, np.ndarray, List[str]]:
        """ksg_snapshot_statuses: (codes[N], message index[N] (-1 = none),
        distinct messages) of every node's Filter status word at once."""
        w = np.ascontiguousarray(words, np.uint32)
        n = len(w)
        code = np.zeros(n, np.int32)
        msg = np.zeros(n, np.int32)
        nm, ln = i32(), i64()
        u32p = C.POINTER(C.c_uint32)
        args = (self.h, pod, w.ctypes.data_as(u32p), n, code.ctypes.data_as(C.POINTER(i32)),
                msg.ctypes.data_as(C.POINTER(i32)))
        buf = getattr(self, "_status_buf", None)
        if buf is None:
            buf = self._status_buf = C.create_string_buffer(1 << 16)
        self._check(self._statuses(*args, buf, len(buf), C.byref(nm), C.byref(ln)), "statuses")
        if ln.value > len(buf):   # one more call with a buffer that fits
            buf = self._status_buf = C.create_string_buffer(ln.value)
            self._check(self._statuses(*args, buf, len(buf), C.byref(nm), C.byref(ln)), "statuses")
        texts = buf.raw[:ln.value].split(b"\0")[:nm.value]
        return code, msg, [t.decode("utf-8") for t in texts]

    def statuses_kept(self, pod: int, words) -> Tuple[np.ndarray, np.ndarray, List[str]]:
        """ksg_snapshot_statuses_kept: ksg_snapshot_statuses into the
        snapshot's own arrays (only the previous and the current rejected
        nodes written when the last call rejected few); returns copies."""
        w = np.ascontiguousarray(words, np.uint32)
        n = len(w)
        pc, pm = C.POINTER(i32)(), C.POINTER(i32)()
        nm, ln = i32(), i64()
        buf = getattr(self, "_status_buf", None)
        if buf is None:
            buf = self._status_buf = C.create_string_buffer(1 << 16)
        args = (self.h, pod, w.ctypes.data_as(C.POINTER(C.c_uint32)), n, C.byref(pc), C.byref(pm))
        self._check(self._statuses_kept(*args, buf, len(buf), C.byref(nm), C.byref(ln)), "statuses_kept")
        if ln.value > len(buf):   # the arrays already hold this call's output; the texts once more
            buf = self._status_buf = C.create_string_buffer(ln.value)
            self._check(self._statuses_kept(*args, buf, len(buf), C.byref(nm), C.byref(ln)), "statuses_kept")
        code = np.ctypeslib.as_array(pc, (n,)).copy() if n else np.zeros(0, np.int32)
        msg = np.ctypeslib.as_array(pm, (n,)).copy() if n else np.zeros(0, np.int32)
        texts = buf.raw[:ln.value].split(b"\0")[:nm.value]
        return code, msg, [t.decode("utf-8") for t in texts]

    def statuses_kept_stats(self) -> Tuple[int, int]:
        """(sparse, dense) ksg_snapshot_statuses_kept calls so far."""
        a, b = i64(), i64()
        self._check(self._kept_stats(self.h, C.byref(a), C.byref(b)), "statuses_kept_stats")
        return a.value, b.value

    def prefilter(self, pod: int, plugin: int, result_status: int = 0):
        """(code, node names or None) of plugin's PreFilter for the pod."""
        code, has, n = i32(), i32(), i32()
        self._check(self._prefilter(self.h, pod, plugin, result_status, C.byref(code), C.byref(has), None, 0,
                                    C.byref(n)), "prefilter")
        names = None
        if has.value:
            arr = (cp * max(n.value, 1))()
            self._check(self._prefilter(self.h, pod, plugin, result_status, C.byref(code), C.byref(has), arr,
                                        n.value, C.byref(n)), "prefilter")
            names = [arr[i].decode("utf-8") for i in range(n.value)]
        return code.value, names
