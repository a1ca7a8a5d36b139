"""Snapshot / record ingest: quantities, object
conversion, scheduler-config profiles, and round trips generator -> k8s JSON
-> ingest -> identical SoA encoding and identical placements."""
import json
from fractions import Fraction

import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
I = pkg("ingest")
P = pkg("profile")
m = pkg("model")


@pytest.mark.parametrize("s,milli,val", [
    ("100m", 100, 1), ("0.5", 500, 1), ("4", 4000, 4), ("1Gi", 2 ** 30 * 1000, 2 ** 30),
    ("16Gi", 16 * 2 ** 30 * 1000, 16 * 2 ** 30), ("1.5Gi", 3 * 2 ** 29 * 1000, 3 * 2 ** 29),
    ("1G", 10 ** 12, 10 ** 9), ("2k", 2 * 10 ** 6, 2000), ("1e3", 10 ** 6, 1000), ("0.0001", 1, 1),
    ("1.0001m", 2, 1), ("200Mi", 200 * 2 ** 20 * 1000, 200 * 2 ** 20), ("110", 110000, 110), (".5", 500, 1),
    ("5E-3", 5, 1), ("-1", -1000, -1), ("+3", 3000, 3), (3, 3000, 3),
])
def test_parse_quantity(s, milli, val):
    q = I.parse_quantity(s)
    assert I.milli_value(q) == milli
    assert I.value(q) == val


@pytest.mark.parametrize("bad", ["", "m", "1.2.3", "1Qi", "abc", "1 Gi"])
def test_parse_quantity_rejects(bad):
    with pytest.raises(ValueError):
        I.parse_quantity(bad)


def test_readme_templates():
    """The web UI's node/pod templates (web/components/lib/templates/node.yaml,
    pod.yaml), i.e. the README example's objects, as ingested."""
    node = I.node_from_k8s({"metadata": {"name": "node-282x7", "labels": {}}, "spec": {},
                            "status": {"capacity": {"cpu": "4", "memory": "32Gi", "pods": "110"},
                                       "allocatable": {"cpu": "4", "memory": "32Gi", "pods": "110"}}})
    assert node.allocatable == {"cpu": 4000, "memory": 32 * 2 ** 30, "pods": 110}
    pod = I.pod_from_k8s({"metadata": {"name": "hoge-pod", "namespace": "default", "labels": {}},
                          "spec": {"containers": [{"name": "pause", "image": "registry.k8s.io/pause:3.5",
                                                   "resources": {"limits": {"cpu": "100m", "memory": "16Gi"},
                                                                 "requests": {"cpu": "100m", "memory": "16Gi"}}}]}})
    assert m.pod_requests(pod) == {"cpu": 100, "memory": 16 * 2 ** 30}


def test_limits_default_requests():
    pod = I.pod_from_k8s({"metadata": {"name": "p"}, "spec": {"containers": [
        {"resources": {"limits": {"cpu": "2", "example.com/fpga": "1"}, "requests": {"cpu": "1"}}}]}})
    assert pod.containers[0].requests == {"cpu": 1000, "example.com/fpga": 1}


def test_profile_from_config_multipoint_merge():
    cfg = {"profiles": [{"plugins": {"multiPoint": {
        "enabled": [{"name": "NodeResourcesFit", "weight": 5}, {"name": "ImageLocality", "weight": 3}],
        "disabled": [{"name": "TaintToleration"}]}},
        "pluginConfig": [{"name": "NodeResourcesFit", "args": {"scoringStrategy": {
            "type": "MostAllocated", "resources": [{"name": "cpu", "weight": 2}, {"name": "memory", "weight": 1}]}}},
            {"name": "InterPodAffinity", "args": {"hardPodAffinityWeight": 4}}]}],
        "percentageOfNodesToScore": 100}
    prof, pct = I.profile_from_config(cfg)
    names = [n for n, _ in prof.plugins]
    assert "TaintToleration" not in names
    assert dict(prof.plugins)["NodeResourcesFit"] == 5 and dict(prof.plugins)["ImageLocality"] == 3
    # re-configured defaults keep their default position (mergePluginSet)
    assert names.index("NodeResourcesFit") < names.index("VolumeRestrictions")
    assert prof.fit_strategy == P.MOST_ALLOCATED and prof.fit_resources == [("cpu", 2), ("memory", 1)]
    assert prof.hard_pod_affinity_weight == 4 and pct == 100
    assert prof.weights()["NodeResourcesFit"] == 5


def test_profile_from_config_refuses_unmodelled():
    # RequestedToCapacityRatio without a shape: the scheduler's validation refuses it
    with pytest.raises(ValueError):
        I.profile_from_config({"profiles": [{"pluginConfig": [{"name": "NodeResourcesFit", "args": {
            "scoringStrategy": {"type": "RequestedToCapacityRatio"}}}]}]})
    with pytest.raises(ValueError):
        I.profile_from_config({"profiles": [{"plugins": {"multiPoint": {"enabled": [{"name": "NodeNumber"}]}}}]})


def test_profile_from_config_rtcr_and_default_constraints():
    """RequestedToCapacityRatio's shape and PodTopologySpread defaultingType
    List with defaultConstraints are read, validated and written back."""
    cfg = {"profiles": [{"pluginConfig": [
        {"name": "NodeResourcesFit", "args": {"scoringStrategy": {
            "type": "RequestedToCapacityRatio", "resources": [{"name": "cpu", "weight": 3}],
            "requestedToCapacityRatio": {"shape": [{"utilization": 0, "score": 0},
                                                   {"utilization": 100, "score": 10}]}}}},
        {"name": "PodTopologySpread", "args": {"defaultingType": "List", "defaultConstraints": [
            {"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule"},
            {"maxSkew": 2, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "ScheduleAnyway"}]}}]}],
        "percentageOfNodesToScore": 100}
    prof, _ = I.profile_from_config(cfg)
    assert prof.fit_strategy == P.REQUESTED_TO_CAPACITY_RATIO and prof.fit_shape == [(0, 0), (100, 10)]
    assert not prof.pts_system_defaulted
    assert [(c.max_skew, c.topology_key, c.when_unsatisfiable) for c in prof.pts_default_constraints] == [
        (1, "topology.kubernetes.io/zone", "DoNotSchedule"), (2, "kubernetes.io/hostname", "ScheduleAnyway")]
    back, _ = I.profile_from_config(I.profile_to_config(prof))
    assert back.fit_shape == prof.fit_shape and back.pts_default_constraints == prof.pts_default_constraints
    bad = [
        ("NodeResourcesFit", {"scoringStrategy": {"type": "RequestedToCapacityRatio", "requestedToCapacityRatio": {
            "shape": [{"utilization": 50, "score": 1}, {"utilization": 40, "score": 2}]}}}),
        ("NodeResourcesFit", {"scoringStrategy": {"type": "RequestedToCapacityRatio", "requestedToCapacityRatio": {
            "shape": [{"utilization": 0, "score": 11}]}}}),
        ("PodTopologySpread", {"defaultingType": "System", "defaultConstraints": [
            {"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule"}]}),
        ("PodTopologySpread", {"defaultingType": "List", "defaultConstraints": [
            {"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule",
             "labelSelector": {"matchLabels": {"a": "b"}}}]}),
        ("PodTopologySpread", {"defaultingType": "List", "defaultConstraints": [
            {"maxSkew": 0, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule"}]}),
    ]
    for name, args in bad:
        with pytest.raises(ValueError):
            I.profile_from_config({"profiles": [{"pluginConfig": [{"name": name, "args": args}]}]})


def _same_encoding(a, b):
    assert a.cluster.node_names == b.cluster.node_names
    assert sorted(a.cluster.arrays) == sorted(b.cluster.arrays)
    for k in a.cluster.arrays:
        np.testing.assert_array_equal(a.cluster.arrays[k], b.cluster.arrays[k], err_msg=k)
    np.testing.assert_array_equal(a.workload.pods, b.workload.pods)
    np.testing.assert_array_equal(a.workload.prog, b.workload.prog)


ROUND_TRIP = {
    "readme-kat": G.readme_kat,
    "c1": lambda: G.config1(n_nodes=40, n_pods=120),
    "c2": lambda: G.config2(n_nodes=60, n_pods=150, seed=21),
    "c2-most": lambda: (lambda n, p, _: (n, p, P.config2_profile(strategy=P.MOST_ALLOCATED)))(
        *G.config2(n_nodes=50, n_pods=80, seed=12)),
    "c3": lambda: G.config3(n_nodes=40, n_pods=150, apps=8, zones=4),
    "c5": lambda: G.config5(n_nodes=60, n_pods=40, n_images=50, taint_vocab=64, taints_per_node=8,
                            images_per_node=10),
}


@pytest.mark.parametrize("name", sorted(ROUND_TRIP))
def test_snapshot_round_trip(name):
    import binding
    nodes, pods, prof = ROUND_TRIP[name]()
    doc = json.loads(json.dumps(I.snapshot_document(nodes, pods, prof)))
    snap = I.load_snapshot(doc)
    assert not snap.bound and snap.queue == list(range(len(pods)))
    assert snap.profile.plugins == prof.plugins
    direct = E.Encoder(nodes, pods, prof)
    via = E.Encoder(snap.nodes, snap.pods, snap.profile)
    _same_encoding(direct, via)
    o = binding.Oracle(2)
    o.load(via, E.encode_profile(snap.profile, via.cluster.res_names))
    pl_via, _ = o.run_queue(0, len(pods))
    o.load(direct, E.encode_profile(prof, direct.cluster.res_names))
    pl_direct, _ = o.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl_via, pl_direct)


def test_bound_pods_and_priority_order():
    nodes, pods, prof = G.config2(n_nodes=20, n_pods=30, seed=4)
    doc = I.snapshot_document(nodes, pods, prof)
    doc["pods"][3]["spec"]["nodeName"] = nodes[5].name        # already running
    doc["pods"][7]["spec"]["nodeName"] = "gone-node"           # bound to a node not in the snapshot
    doc["pods"][10]["spec"]["priority"] = 100
    doc["priorityClasses"] = [{"metadata": {"name": "hi"}, "value": 50}]
    doc["pods"][12]["spec"]["priorityClassName"] = "hi"
    snap = I.load_snapshot(doc)
    assert snap.bound == [(0, 5)] and snap.pods[0].name == pods[3].name
    assert snap.skipped == [pods[7].name]
    q = [snap.pods[i].name for i in snap.queue]
    assert q[0] == pods[10].name and q[1] == pods[12].name
    assert len(q) == 28


def test_namespace_selector_resolved():
    doc = {"nodes": [], "namespaces": [{"metadata": {"name": "a", "labels": {"team": "x"}}},
                                       {"metadata": {"name": "b", "labels": {"team": "y"}}}],
           "pods": [{"metadata": {"name": "p", "namespace": "a"}, "spec": {"containers": [{}], "affinity": {
               "podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                   {"labelSelector": {"matchLabels": {"app": "z"}}, "topologyKey": "zone",
                    "namespaceSelector": {"matchLabels": {"team": "y"}}},
                   {"labelSelector": {"matchLabels": {"app": "z"}}, "topologyKey": "zone",
                    "namespaceSelector": {"matchLabels": {"team": "none"}}}]}}}}]}
    snap = I.load_snapshot(doc)
    t0, t1 = snap.pods[0].pod_affinity_required
    assert t0.namespaces == ("b",) and t0.namespace_selector is None
    assert t1.namespaces == (I.NO_NAMESPACE,)


def test_replay_records():
    nodes, pods, prof = G.config1(n_nodes=5, n_pods=6)
    doc = I.snapshot_document(nodes, pods, prof)
    recs = [{"time": "t", "event": "Add", "resource": o} for o in doc["nodes"] + doc["pods"]]
    upd = json.loads(json.dumps(doc["nodes"][1]))
    upd["metadata"]["labels"]["extra"] = "1"
    recs.append({"time": "t", "event": "Update", "resource": upd})
    recs.append({"time": "t", "event": "Delete", "resource": doc["pods"][2]})
    out = I.replay_records(json.dumps(recs))
    assert [n["metadata"]["name"] for n in out["nodes"]] == [n.name for n in nodes]
    assert out["nodes"][1]["metadata"]["labels"]["extra"] == "1"
    assert [p["metadata"]["name"] for p in out["pods"]] == [p.name for i, p in enumerate(pods) if i != 2]
    snap = I.load_snapshot(out)
    assert len(snap.queue) == 5


def test_snapshot_with_running_pods_end_to_end():
    """A snapshot whose first pods already run: the mirror (C++ oracle engine,
    native serialiser) and the Python restatement agree on every annotation."""
    import binding
    import pyoracle
    F = pkg("framework")
    A = pkg("annotations")
    nodes, pods, prof = G.config3(n_nodes=30, n_pods=90, apps=6, zones=3)
    doc = I.snapshot_document(nodes, pods, prof)
    for k in range(30):                      # the first 30 pods already run, round robin
        doc["pods"][k]["spec"]["nodeName"] = nodes[k % len(nodes)].name
    snap = I.load_snapshot(doc)
    assert len(snap.bound) == 30 and len(snap.queue) == 60
    s = F.DebuggableScheduler(snap.nodes, snap.pods, snap.profile, engine=binding.Oracle(2), bound=snap.bound)
    got = []
    for i in snap.queue:
        s.schedule_one(i)
        got.append(s.annotations(i))
    from helpers import pyoracle_annotations
    bound = [(snap.pods[pi], snap.nodes[ni].name) for pi, ni in snap.bound]
    queue = [snap.pods[i] for i in snap.queue]
    want, _ = pyoracle_annotations(snap.nodes, queue, snap.profile, bound)
    assert want == got
    assert any(a[A.SELECTED_NODE] for a in got)


# ---- the reference's own export sample (simulator/docs/api-samples/v1/export.md) ----

def _export(case):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "export_md.json")) as f:
        return json.load(f)[case]


LEGACY = ("EBSLimits", "GCEPDLimits", "AzureDiskLimits")


def export_config_loadable():
    """case 1's schedulerConfig without the three volume-limit plugins the
    simulator's registry (in-tree MultiPoint names only, plugins.go:39-60)
    does not hold."""
    import copy
    cfg = copy.deepcopy(_export("case1")["schedulerConfig"])
    flt = cfg["profiles"][0]["plugins"]["filter"]
    flt["enabled"] = [e for e in flt["enabled"] if e["name"] not in LEGACY]
    return cfg


@pytest.mark.parametrize("case", ["case1", "case2"])
def test_export_sample_refused_like_the_registry(case):
    """Both samples name EBSLimits / GCEPDLimits / AzureDiskLimits under
    filter; the simulator registers only the in-tree MultiPoint plugins, so
    its framework cannot be built from this configuration either."""
    with pytest.raises(ValueError, match="EBSLimits"):
        I.load_snapshot(_export(case))


def test_export_sample_priority_classes_and_empty_cluster():
    doc = _export("case2")
    doc["schedulerConfig"] = export_config_loadable()
    snap = I.load_snapshot(doc)
    assert snap.nodes == [] and snap.pods == [] and snap.queue == []


def test_export_sample_per_point_expansion():
    """The per-point sets of the sample expanded against the in-tree
    MultiPoint set (profile.py docstring); weights: the framework takes the
    Score point's own, the store map MultiPoint's."""
    prof, pct = I.profile_from_config(export_config_loadable())
    assert pct == 0
    nm = lambda ids: [P.PLUGIN_NAMES[i] for i in ids]
    assert nm(prof.filter_order()) == [
        "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
        "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread",
        "InterPodAffinity"]
    assert nm(prof.prefilter_order()) == [
        "NodeResourcesFit", "NodePorts", "VolumeRestrictions", "PodTopologySpread", "InterPodAffinity",
        "VolumeBinding", "NodeAffinity", "NodeVolumeLimits", "VolumeZone"]
    assert nm(prof.prescore_order()) == [
        "InterPodAffinity", "PodTopologySpread", "TaintToleration", "NodeAffinity", "NodeResourcesFit",
        "VolumeBinding", "NodeResourcesBalancedAllocation"]
    assert nm(prof.score_order()) == [
        "NodeResourcesBalancedAllocation", "ImageLocality", "InterPodAffinity", "NodeResourcesFit",
        "NodeAffinity", "PodTopologySpread", "TaintToleration", "VolumeBinding"]
    sel, store = prof.selection_weights(), prof.weights()
    for k, v in {"TaintToleration": 1, "NodeAffinity": 1, "PodTopologySpread": 2, "InterPodAffinity": 1,
                 "NodeResourcesFit": 1, "NodeResourcesBalancedAllocation": 1, "ImageLocality": 1}.items():
        assert sel[k] == v, k
    for k, v in {"TaintToleration": 3, "NodeAffinity": 2, "PodTopologySpread": 2, "InterPodAffinity": 2,
                 "NodeResourcesFit": 1, "NodeResourcesBalancedAllocation": 1, "ImageLocality": 1}.items():
        assert store[k] == v, k
    assert prof.hard_pod_affinity_weight == 1 and prof.fit_strategy == P.LEAST_ALLOCATED


def test_per_point_disable_and_errors():
    prof, _ = I.profile_from_config({"profiles": [{"plugins": {"filter": {"disabled": [{"name": "NodeAffinity"}]}}}]})
    assert "NodeAffinity" not in [P.PLUGIN_NAMES[i] for i in prof.filter_order()]
    assert "NodeAffinity" in [P.PLUGIN_NAMES[i] for i in prof.score_order()]
    prof, _ = I.profile_from_config({"profiles": [{"plugins": {"score": {
        "enabled": [{"name": "ImageLocality", "weight": 7}], "disabled": [{"name": "*"}]}}}]})
    assert prof.score_order() == [P.IMAGE_LOCALITY] and prof.selection_weights()["ImageLocality"] == 7
    assert prof.weights()["ImageLocality"] == 1          # the store map: MultiPoint's weight wins
    with pytest.raises(ValueError, match="does not extend"):
        I.profile_from_config({"profiles": [{"plugins": {"filter": {"enabled": [{"name": "ImageLocality"}]}}}]})


def test_export_profile_cpp_oracle_vs_pyoracle():
    """The export sample's profile on a small config-3 cluster: the C++
    oracle (selection on the Score point's weights, through encode_profile)
    and pyoracle give the same annotation bytes (store weights = MultiPoint's)."""
    import binding
    from helpers import pyoracle_annotations
    F = pkg("framework")
    nodes, pods, _ = G.config3(n_nodes=30, n_pods=90, apps=6, zones=3)
    doc = I.snapshot_document(nodes, pods, P.default_profile())
    doc["schedulerConfig"] = export_config_loadable()
    snap = I.load_snapshot(doc)
    s = F.DebuggableScheduler(snap.nodes, snap.pods, snap.profile, engine=binding.Oracle(2))
    got = []
    for i in snap.queue:
        s.schedule_one(i)
        got.append(s.annotations(i))
    want, _ = pyoracle_annotations(snap.nodes, [snap.pods[i] for i in snap.queue], snap.profile)
    assert want == got
    # the two weight maps really differ here, so the test separates them
    assert snap.profile.weights()["TaintToleration"] != snap.profile.selection_weights()["TaintToleration"]


# ---- volumes: export.md case 2 holds 2 PVs and 1 PVC ----

def _volume_doc(disable_volume_plugins: bool = False):
    """export.md case 2 (its PVs, PVC and priority classes) plus one node, a
    pod claiming the sample's pvc1 and a pod with only an emptyDir."""
    import copy
    doc = copy.deepcopy(_export("case2"))
    cfg = export_config_loadable()
    if disable_volume_plugins:
        for point in ("multiPoint", "preFilter", "filter"):
            ps = cfg["profiles"][0]["plugins"].setdefault(point, {})
            ps["enabled"] = [e for e in ps.get("enabled") or () if e["name"] not in
                             ("VolumeBinding", "VolumeZone", "NodeVolumeLimits", "VolumeRestrictions")]
            ps["disabled"] = list(ps.get("disabled") or ()) + [
                {"name": n} for n in ("VolumeBinding", "VolumeZone", "NodeVolumeLimits", "VolumeRestrictions")]
    doc["schedulerConfig"] = cfg
    node = I.node_to_k8s(m.Node(name="n1", labels={"kubernetes.io/hostname": "n1"},
                                allocatable={m.CPU: 4000, m.MEMORY: 8 << 30, "pods": 110}))
    def pod(name, volumes):
        d = I.pod_to_k8s(m.Pod(name=name, containers=[m.Container(requests={m.CPU: 100})]))
        d["spec"]["volumes"] = volumes
        return d
    doc["nodes"] = [node]
    doc["pods"] = [pod("scratch", [{"name": "tmp", "emptyDir": {}}]),
                   pod("claims", [{"name": "data", "persistentVolumeClaim": {"claimName": "pvc1"}}])]
    return doc


def test_volumes_parsed_from_the_export_sample():
    doc = _volume_doc()
    assert len(doc["pvs"]) == 2 and len(doc["pvcs"]) == 1 and doc["pvcs"][0]["metadata"]["name"] == "pvc1"
    snap = I.load_snapshot(doc)
    byname = {p.name: p for p in snap.pods}
    assert byname["claims"].volumes == [("data", "persistentVolumeClaim", "pvc1")]
    assert byname["claims"].claim_names() == ["pvc1"]
    assert byname["claims"].volumes_needing_plugins() == []    # claims are modelled (round 5)
    assert byname["scratch"].volumes == [("tmp", "emptyDir", "")]
    assert byname["scratch"].volumes_needing_plugins() == []
    st = byname["claims"].storage
    pvc = st.claim("default", "pvc1")
    assert pvc.volume_name == "pv1" and pvc.fully_bound() and pvc.storage_class == ""
    assert st.pvs["pv1"].claim_ref == ("default", "pvc1") and st.pvs["pv1"].source == "hostPath"
    assert st.pvs["pv2"].claim_ref is None and st.pvs["pv1"].node_affinity is None


def test_claim_volume_encoded_by_python_and_native():
    """A PVC makes the volume plugins' PreFilter run upstream: both encoders
    model them (a volume program) and produce the same bytes; the native one
    resolves the claim against the storage objects added through the C ABI."""
    S = pkg("snapshot")
    snap = I.load_snapshot(_volume_doc())
    enc = E.Encoder(snap.nodes, snap.pods, snap.profile)
    rec = {n: enc.workload.pods[i] for i, n in enumerate(enc.workload.names)}
    assert int(rec["default/claims"]["vol"]) >= 0 and int(rec["default/scratch"]["vol"]) == -1
    fskip = int(rec["default/claims"]["filter_skip"])
    for v in (P.VOLUME_RESTRICTIONS, P.NODE_VOLUME_LIMITS, P.VOLUME_BINDING):
        assert not fskip >> v & 1
    assert fskip >> P.VOLUME_ZONE & 1   # pv1 has no zone labels: VolumeZone's PreFilter Skip
    s = S.Snapshot(snap.profile, snap.nodes, snap.pods)
    s.encode()
    got = s.arrays()
    assert got["pods"].tobytes() == enc.workload.pods.tobytes()
    np.testing.assert_array_equal(got["prog"], enc.workload.prog)


def test_volume_sources_the_plugins_skip_encode():
    """emptyDir (and every source outside the refused set) is the volume
    plugins' Skip; with the volume plugins disabled a claim is irrelevant."""
    snap = I.load_snapshot(_volume_doc())
    pods = [p for p in snap.pods if p.name == "scratch"]
    enc = E.Encoder(snap.nodes, pods, snap.profile)
    fskip = int(enc.workload.pods[0]["filter_skip"])
    for v in (P.VOLUME_RESTRICTIONS, P.NODE_VOLUME_LIMITS, P.VOLUME_BINDING, P.VOLUME_ZONE):
        assert fskip >> v & 1
    snap2 = I.load_snapshot(_volume_doc(disable_volume_plugins=True))
    E.Encoder(snap2.nodes, snap2.pods, snap2.profile)   # no refusal
    S = pkg("snapshot")
    s = S.Snapshot(snap2.profile, snap2.nodes)
    for p in snap2.pods:
        s.add_pod(p)


def test_volume_without_a_source_is_empty_dir():
    """a volume with only a name is an emptyDir after API defaulting
    (SetDefaults_Volume), not an error."""
    doc = _volume_doc()
    doc["pods"][0]["spec"]["volumes"] = [{"name": "bare"}]
    snap = I.load_snapshot(doc)
    byname = {p.name: p for p in snap.pods}
    assert byname["scratch"].volumes == [("bare", "emptyDir", "")]
    assert byname["scratch"].volumes_needing_plugins() == []
