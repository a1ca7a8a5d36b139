"""NodePorts (the Filter plugins on the path) with host
ports: the encoded conflict sets, the C++ oracle, the native snapshot encoder
and (-m gpu) the device's per-node UsedPorts bitmap, each against the pure
Python restatement (oracle/pyoracle.py: HostPortInfo.CheckConflict / Add /
Remove over the node's pods).

Upstream semantics restated [nodeports/node_ports.go, framework/types.go
HostPortInfo; v1.32, not vendored in the reference — DESIGN.md §9]: a pod's
host ports are those of its containers and of its restartable init
containers (GetHostPorts); "" host IP means 0.0.0.0 and "" protocol TCP;
two ports conflict when protocol and port match and either IP is 0.0.0.0 or
the IPs are equal; a pod without host ports is Skipped at PreFilter; the
rejection is Unschedulable with "node(s) didn't have free ports for the
requested pod ports".  Parity with Go itself is unpinned (no reference
fixture holds a hostPort pod)."""
import json

import numpy as np
import pytest

from conftest import pkg
from helpers import pyoracle_annotations

G = pkg("generator")
E = pkg("encoder")
F = pkg("framework")
P = pkg("profile")
PR = pkg("preemption")
S = pkg("snapshot")
I = pkg("ingest")
A = pkg("annotations")
m = pkg("model")
native = pkg("native")

GI = 1024 ** 3
MSG = "node(s) didn't have free ports for the requested pod ports"


def _pod(name, ports=(), node="", init=None):
    p = m.Pod(name=name, containers=[m.Container(image="pause", requests={m.CPU: 100, m.MEMORY: GI},
                                                  host_ports=tuple(ports))],
              init_containers=[init] if init else [])
    p.node_name = node
    return p


def _one_node():
    return [m.Node(name="n0", labels={m.LABEL_HOSTNAME: "n0"},
                   allocatable={m.CPU: 8000, m.MEMORY: 32 * GI, m.EPHEMERAL: 100 * GI, m.PODS: 110})]


# (running pod's ports, candidate's ports, conflict?) — HostPortInfo.CheckConflict
RULES = [
    ([("127.0.0.1", "TCP", 8080)], [("", "TCP", 8080)], True),             # bind-all vs specific
    ([("", "TCP", 8080)], [("127.0.0.1", "TCP", 8080)], True),             # specific vs bind-all
    ([("127.0.0.1", "TCP", 8080)], [("10.0.0.1", "TCP", 8080)], False),    # two specific IPs
    ([("127.0.0.1", "TCP", 8080)], [("127.0.0.1", "", 8080)], True),       # "" protocol = TCP
    ([("", "UDP", 53)], [("", "TCP", 53)], False),                         # protocol differs
    ([("", "TCP", 80)], [("", "TCP", 81)], False),
    ([("0.0.0.0", "TCP", 80)], [("", "TCP", 80)], True),
    ([], [("", "TCP", 80)], False),
]


def _verdicts(engine_name):
    """Filter verdict of each RULES candidate on n0, with the running pod bound."""
    import binding
    import pyoracle
    out = []
    for run, cand, _ in RULES:
        nodes = _one_node()
        running = _pod("run", run, node="n0")
        pods = [running, _pod("cand", cand)]
        if engine_name == "pyoracle":
            r = pyoracle.run_queue(nodes, [(running, "n0")], pods[1:], P.default_profile())[0]
            out.append(r["filter"]["n0"].get("NodePorts"))
        else:
            s = F.DebuggableScheduler(nodes, pods, P.default_profile(), engine=binding.Oracle(1), bound=[(0, 0)])
            s.schedule_one(1)
            flt = json.loads(s.annotations(1)[A.FILTER])
            out.append(flt["n0"].get("NodePorts"))
    return out


@pytest.mark.parametrize("engine", ["pyoracle", "oracle_cpp"])
def test_conflict_rules(engine):
    got = _verdicts(engine)
    for (run, cand, conflict), v in zip(RULES, got):
        assert v == (MSG if conflict else "passed"), (run, cand, v)


def test_host_ports_of_a_pod():
    """GetHostPorts: restartable init containers count, plain init containers
    and hostPort 0 do not."""
    side = _pod("s", init=m.Container(image="envoy", restartable=True, host_ports=(("", "TCP", 15000),)))
    init = _pod("i", init=m.Container(image="busybox", host_ports=(("", "TCP", 15000),)))
    zero = _pod("z", [("", "TCP", 0)])
    assert side.host_ports() == [("", "TCP", 15000)]
    assert init.host_ports() == [] and zero.host_ports() == []
    enc = E.Encoder(_one_node(), [side, init, zero], P.default_profile())
    pods = enc.workload.pods
    assert pods["ports"][0] >= 0 and pods["ports"][1] == -1 and pods["ports"][2] == -1
    # PreFilter Skip without host ports
    assert not (pods["filter_skip"][0] >> P.NODE_PORTS) & 1
    assert (pods["filter_skip"][1] >> P.NODE_PORTS) & 1


def _framework(engine, nodes, pods, bound, prof):
    s = F.DebuggableScheduler(nodes, pods, prof, engine=engine, bound=bound)
    nb = len(bound)
    placed = [s.schedule_one(i) for i in range(nb, len(pods))]
    return placed, [s.annotations(i) for i in range(nb, len(pods))]


def _check_case(engine, nodes, pods, bound, prof):
    nb = len(bound)
    placed, ann = _framework(engine, nodes, pods, bound, prof)
    want, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert [r["selected_index"] for r in recs] == placed
    for k, (w, g) in enumerate(zip(want, ann)):
        assert w == g, f"pod {pods[nb + k].name}: annotations differ"
    return placed, ann


@pytest.mark.parametrize("seed", [9, 10])
def test_daemonset_case_oracle_vs_pyoracle(seed):
    import binding
    nodes, pods, bound, prof = G.host_ports_case(seed=seed)
    placed, ann = _check_case(binding.Oracle(2), nodes, pods, bound, prof)
    rejected = sum(MSG in a[A.FILTER] for a in ann)
    assert rejected > 20 and -1 in placed      # ports ran out on every node for some pods


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_zoo_with_ports_oracle_vs_pyoracle(seed):
    import binding
    from zoo import zoo
    nodes, pods, prof = zoo(seed, ports=True)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    placed, got = _framework(binding.Oracle(2), nodes, pods, [], prof)
    assert want == got
    assert any(MSG in a[A.FILTER] for a in got)


def _daemonset_document(n_nodes=12, n_queue=60, seed=3):
    """A cluster snapshot as the simulator exports it: node-exporter pods
    owned by a DaemonSet, already running on every node with hostPort 9100,
    pinned by the controller's matchFields node affinity, then a queue."""
    nodes, pods, _, prof = G.host_ports_case(n_nodes=n_nodes, n_queue=n_queue, seed=seed, daemonset=False)
    doc = I.snapshot_document(nodes, pods, prof)
    for i, nd in enumerate(nodes):
        doc["pods"].insert(i, {
            "metadata": {"name": f"node-exporter-{i:03d}", "namespace": "monitoring",
                         "ownerReferences": [{"kind": "DaemonSet", "name": "node-exporter", "controller": True}]},
            "spec": {"nodeName": nd.name,
                     "containers": [{"name": "exporter", "image": "prom/node-exporter",
                                     "resources": {"requests": {"cpu": "50m", "memory": "64Mi"}},
                                     "ports": [{"containerPort": 9100, "hostPort": 9100, "protocol": "TCP"}]}],
                     "tolerations": [{"operator": "Exists"}],
                     "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                         "nodeSelectorTerms": [{"matchFields": [
                             {"key": "metadata.name", "operator": "In", "values": [nd.name]}]}]}}}}})
    return json.loads(json.dumps(doc))


def test_ingested_daemonset_pods():
    import binding
    snap = I.load_snapshot(_daemonset_document())
    assert len(snap.bound) == 12
    assert snap.pods[0].host_ports() == [("", "TCP", 9100)]
    s = F.DebuggableScheduler(snap.nodes, snap.pods, snap.profile, engine=binding.Oracle(2), bound=snap.bound)
    got = []
    for i in snap.queue:
        s.schedule_one(i)
        got.append(s.annotations(i))
    bound = [(snap.pods[pi], snap.nodes[ni].name) for pi, ni in snap.bound]
    want, _ = pyoracle_annotations(snap.nodes, [snap.pods[i] for i in snap.queue], snap.profile, bound)
    assert want == got
    exporters = [a for i, a in zip(snap.queue, got) if snap.pods[i].name.startswith("exporter-")]
    assert exporters and all(a[A.SELECTED_NODE] == "" for a in exporters)   # 9100 taken everywhere


def test_native_snapshot_encodes_host_ports(built):
    """The native encoder: byte-identical to encoder.py with bound DaemonSet
    pods; appended pods reuse the port vocabulary (frozen append) unless they
    bring a new port (full re-encode) — both equal to one full encode."""
    nodes, pods, bound, prof = G.host_ports_case(n_nodes=20, n_queue=120)
    enc = E.Encoder(nodes, pods, prof)
    snap = S.Snapshot(prof, nodes, pods, bound)
    snap.encode()
    got = snap.arrays()
    assert got["pods"].tobytes() == enc.workload.pods.tobytes()
    np.testing.assert_array_equal(got["prog"], enc.workload.prog)
    assert got["meta"]["n_port_vocab"] == len(enc.port_vocab) > 0
    split = len(pods) - 30
    for extra, appended_want in ((None, 1), (_pod("new-port", [("", "TCP", 31337)]), 0)):
        ps = list(pods) + ([extra] if extra else [])
        full = S.Snapshot(prof, nodes, ps, bound)
        full.encode()
        inc = S.Snapshot(prof, nodes, ps[:split], bound)
        inc.encode()
        for p in ps[split:]:
            inc.add_pod(p)
        assert inc.encode_incremental() == appended_want
        a, b = inc.arrays(), full.arrays()
        assert a["pods"].tobytes() == b["pods"].tobytes()
        np.testing.assert_array_equal(a["prog"], b["prog"])


def test_native_status_message(built):
    nodes = _one_node()
    pods = [_pod("run", [("", "TCP", 80)], node="n0"), _pod("cand", [("", "TCP", 80)])]
    snap = S.Snapshot(P.default_profile(), nodes, pods, [(0, 0)])
    snap.encode()
    word = P.NODE_PORTS + 1
    code, msg = snap.status(1, word, 0)
    assert code == F.Status.UNSCHEDULABLE and msg == MSG


@pytest.mark.parametrize("engine", ["oracle", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_preemptor_with_host_ports_kat(engine, request):
    """Worked by hand: n0 runs "low" (priority 0, hostPort 80) and "keep"
    (priority 0, hostPort 81); "high" (priority 100) wants 80.  NodePorts
    rejects n0 (Unschedulable: preemption may help); the dry run removes both
    lower-priority pods, reprieves "low" first (the more important by name
    order at equal priority and start) -- 80 is then held again, so "low"
    stays evicted -- then "keep", which fits.  One victim, "low"; the retry
    binds "high" on n0.  (Round 5 refused every preemptor with host ports.)"""
    import binding
    nodes = _one_node()
    low, keep = _pod("low", [("", "TCP", 80)], node="n0"), _pod("keep", [("", "TCP", 81)], node="n0")
    cand = _pod("high", [("", "TCP", 80)])
    low.priority = keep.priority = 0
    cand.priority = 100
    pods = [low, keep, cand]
    assert not PR.needs_static_verdict(P.default_profile(), cand)   # no claims: the dry run decides alone
    eng = binding.Oracle(1) if engine == "oracle" else (request.getfixturevalue("built") and native.Engine(device=0))
    s = F.DebuggableScheduler(nodes, pods, P.default_profile(), engine=eng, bound=[(0, 0), (1, 0)])
    placed = s.schedule_one(2)
    (pi, nom, victims), = s.preemptions
    assert (pi, nom, [pods[v].name for v in victims]) == (2, 0, ["low"])
    assert placed == 0


# ---- GPU: the UsedPorts bitmap on the device -------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("seed", [9, 10])
def test_gpu_daemonset_case_matches_pyoracle(built, seed):
    nodes, pods, bound, prof = G.host_ports_case(seed=seed)
    placed, ann = _check_case(native.Engine(device=0), nodes, pods, bound, prof)
    assert sum(MSG in a[A.FILTER] for a in ann) > 20


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_zoo_with_ports_matches_pyoracle(built, seed):
    from zoo import zoo
    nodes, pods, prof = zoo(seed, ports=True)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    _, got = _framework(native.Engine(device=0), nodes, pods, [], prof)
    assert want == got


@pytest.mark.gpu
def test_gpu_run_queue_with_ports_matches_oracle(built):
    """The whole queue in one ksg_run_queue (the batched paths refuse a range
    with host ports; the queue kernel models UsedPorts) against the C++
    oracle, larger than the annotation cases."""
    import binding
    nodes, pods, bound, prof = G.host_ports_case(n_nodes=300, n_queue=3000, seed=12)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    out = []
    for eng in (native.Engine(device=0), binding.Oracle(4)):
        eng.load(enc, pf)
        for pi, ni in bound:
            eng.commit(pi, ni)
        pl, res = eng.run_queue(len(bound), len(pods) - len(bound))
        out.append((np.asarray(pl).copy(), res["n_feasible"].copy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert (out[0][0] == -1).any() and (out[0][0] >= 0).sum() > 1000


@pytest.mark.gpu
def test_gpu_ingested_daemonset_snapshot(built):
    """Ingested DaemonSet pods through the native snapshot (C views) onto the
    device: per-cycle eval + commit against the C++ oracle."""
    import binding
    snap_doc = I.load_snapshot(_daemonset_document(n_nodes=40, n_queue=400))
    snap = S.Snapshot(snap_doc.profile, snap_doc.nodes, snap_doc.pods, snap_doc.bound)
    eng = native.Engine(device=0)
    snap.load(eng)
    enc = E.Encoder(snap_doc.nodes, snap_doc.pods, snap_doc.profile)
    o = binding.Oracle(2)
    o.load(enc, E.encode_profile(snap_doc.profile, enc.cluster.res_names))
    for pi, ni in snap_doc.bound:
        o.commit(pi, ni)
    n_rej = 0
    for i in snap_doc.queue:
        rg, ro = eng.eval(i), o.eval(i)
        assert (rg.selected, rg.n_feasible) == (ro.selected, ro.n_feasible), snap_doc.pods[i].name
        n_rej += rg.selected < 0
        if rg.selected >= 0:
            eng.commit(i, rg.selected)
            o.commit(i, ro.selected)
    assert n_rej > 0
