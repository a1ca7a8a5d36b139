"""DefaultPreemption PostFilter: victim selection,
candidate choice, postfilter-result and the preemptor's retry.

The reference wraps upstream v1.32 DefaultPreemption (wrappedplugin.go:550-583,
store.go:442-458); the plugin source is not vendored, so the hand-worked
known-answer cases below restate its rules (SelectVictimsOnNode reprieve
order, pickOneNodeForPreemption criteria) on inputs small enough to check by
hand, and the generated cases compare the framework (C++ oracle engine on
CPU, libksched.so on the GPU) with the independent pyoracle restatement,
annotation bytes included.  Parity against Go itself is unpinned."""
import json

import numpy as np
import pytest

from conftest import pkg
from helpers import pyoracle_annotations

G = pkg("generator")
F = pkg("framework")
A = pkg("annotations")
P = pkg("profile")
PR = pkg("preemption")
m = pkg("model")
native = pkg("native")

GI = 1024 ** 3


def _kat(a_start: int):
    """node-0: a (prio 1, 2 cores, start a_start) + b (prio 5, 2 cores);
    node-1: c, d (prio 1, 1 core, starts 10, 20) + e (prio 1, 2 cores, start 30);
    node-2: NoSchedule taint.  Each node has 4 cores; the preemptor (prio 10)
    asks for 2.  Worked by hand: node-0 reprieves b, evicts a; node-1
    reprieves c and d, evicts e.  Both: one victim of priority 1, so the
    latest earliest start decides (a_start vs 30)."""
    nodes = []
    for i in range(3):
        nodes.append(m.Node(name=f"node-{i}", labels={m.LABEL_HOSTNAME: f"node-{i}"},
                            allocatable={m.CPU: 4000, m.MEMORY: 16 * GI, m.EPHEMERAL: 100 * GI, m.PODS: 110}))
    nodes[2].taints = [m.Taint("dedicated", "x", m.NO_SCHEDULE)]

    def pod(name, cpu, prio, start=None, node=""):
        p = m.Pod(name=name, containers=[m.Container(image="pause", requests={m.CPU: cpu, m.MEMORY: GI})])
        p.priority, p.start_time, p.node_name = prio, start, node
        return p
    running = [(pod("a", 2000, 1, a_start, "node-0"), 0), (pod("b", 2000, 5, 40, "node-0"), 0),
               (pod("c", 1000, 1, 10, "node-1"), 1), (pod("d", 1000, 1, 20, "node-1"), 1),
               (pod("e", 2000, 1, 30, "node-1"), 1)]
    pods = [p for p, _ in running] + [pod("preemptor", 2000, 10)]
    bound = [(i, n) for i, (_, n) in enumerate(running)]
    return nodes, pods, bound, P.default_profile()


def _oracle_engine():
    import binding
    return binding.Oracle(2)


def _run_framework(engine, nodes, pods, bound, prof):
    s = F.DebuggableScheduler(nodes, pods, prof, engine=engine, bound=bound)
    nb = len(bound)
    placed = [s.schedule_one(i) for i in range(nb, len(pods))]
    return s, placed, [s.annotations(i) for i in range(nb, len(pods))]


@pytest.mark.parametrize("a_start,node,victim", [(100, "node-0", "a"), (20, "node-1", "e")])
def test_kat_victims_and_nomination(a_start, node, victim):
    nodes, pods, bound, prof = _kat(a_start)
    s, placed, ann = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    (pi, nom, victims), = s.preemptions
    assert s.node_names[nom] == node and [pods[v].name for v in victims] == [victim]
    assert s.node_names[placed[0]] == node
    a = ann[0]
    hist = json.loads(a[A.RESULT_HISTORY])
    assert len(hist) == 2                         # the failed attempt, then the retry
    first, retry = hist
    assert json.loads(first[A.POSTFILTER]) == {"node-0": ({"DefaultPreemption": "preemption victim"}
                                                          if node == "node-0" else {}),
                                               "node-1": ({"DefaultPreemption": "preemption victim"}
                                                          if node == "node-1" else {}),
                                               "node-2": {}}
    assert first[A.SELECTED_NODE] == ""
    assert set(json.loads(retry[A.FILTER])) == {node}          # evaluateNominatedNode
    assert json.loads(retry[A.SCORE]) == {} and retry[A.SELECTED_NODE] == node
    ora, recs = pyoracle_annotations(nodes, pods[5:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert recs[0]["first_attempt"]["victims"] == [("default", victim)]
    assert ora == ann


def test_never_policy_and_equal_priority_do_not_preempt():
    nodes, pods, bound, prof = _kat(100)
    pods[-1].preemption_policy = "Never"
    s, placed, ann = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    assert placed == [-1] and not s.preemptions
    assert json.loads(ann[0][A.POSTFILTER]) == {"node-0": {}, "node-1": {}, "node-2": {}}
    nodes, pods, bound, prof = _kat(100)
    pods[-1].priority = 1                  # nothing of strictly lower priority on node-1
    for p in pods[:5]:
        p.priority = max(p.priority, 1)
    s, placed, _ = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    assert placed == [-1] and not s.preemptions


def test_pick_one_node_criteria():
    def v(prio, start=None):
        p = m.Pod(name=f"v{prio}-{start}")
        p.priority, p.start_time = prio, start
        return p
    # lowest highest-priority victim
    assert PR.pick_one_node([(0, [v(5)], 0), (1, [v(3), v(3)], 0)]) == 1
    # then lowest priority sum
    assert PR.pick_one_node([(0, [v(5), v(1)], 0), (1, [v(5)], 0)]) == 1
    # then fewest victims (equal sums impossible with the MaxInt32 offset unless counts match)
    assert PR.pick_one_node([(0, [v(5, 1), v(0, 1)], 0), (1, [v(5, 2), v(0, 2)], 0)]) == 1   # latest start
    # complete tie: lowest node index
    assert PR.pick_one_node([(4, [v(5, 7)], 0), (2, [v(5, 7)], 0)]) == 2
    assert PR.num_candidates(5, P.Profile()) == 5 and PR.num_candidates(5000, P.Profile()) == 500


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_generated_cases_framework_vs_pyoracle(seed):
    nodes, pods, bound, prof = G.preemption_case(seed=seed)
    s, placed, ann = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert len(s.preemptions) > 10
    assert [r["selected_index"] for r in recs] == placed
    pre = [(pi - nb, s.node_names[n], [(pods[v].namespace, pods[v].name) for v in vs]) for pi, n, vs in s.preemptions]
    ref = [(k, r["first_attempt"]["nominated"], r["first_attempt"]["victims"])
           for k, r in enumerate(recs) if "first_attempt" in r]
    assert pre == ref
    assert ann == ora


def test_framework_run_queue_matches_single_cycles():
    nodes, pods, bound, prof = G.preemption_case(seed=8)
    nb = len(bound)
    s1, placed, _ = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    s2 = F.DebuggableScheduler(nodes, pods, prof, engine=_oracle_engine(), bound=bound)
    pl, res = s2.run_queue(nb, len(pods) - nb)
    assert list(pl) == placed and s2.preemptions == s1.preemptions


def _vs_pyoracle(nodes, pods, bound, prof, engine=None):
    s, placed, ann = _run_framework(engine or _oracle_engine(), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert [r["selected_index"] for r in recs] == placed
    pre = [(pi - nb, s.node_names[n], [(pods[v].namespace, pods[v].name) for v in vs]) for pi, n, vs in s.preemptions]
    ref = [(k, r["first_attempt"]["nominated"], r["first_attempt"]["victims"])
           for k, r in enumerate(recs) if "first_attempt" in r]
    assert pre == ref
    assert ann == ora
    return s


def test_static_filter_after_fit_vs_pyoracle():
    """TaintToleration ordered after NodeResourcesFit: node-2 (tainted) holds
    the cheapest victim and its recorded rejection is Fit (Unschedulable),
    but the dry run's TaintToleration still rejects it; the node-static
    verdict (ksg_eval_skipping) keeps it out of the candidates."""
    nodes, pods, bound, prof = _kat(100)
    f = m.Pod(name="f", containers=[m.Container(image="pause", requests={m.CPU: 4000, m.MEMORY: GI})])
    f.priority, f.start_time, f.node_name = 0, 5, "node-2"
    pods.insert(5, f)
    bound.append((5, 2))
    names = [n for n, _ in prof.plugins]
    i, j = names.index("TaintToleration"), names.index("NodeResourcesFit")
    prof.plugins[i], prof.plugins[j] = prof.plugins[j], prof.plugins[i]
    assert PR.needs_static_verdict(prof, pods[-1])
    s = _vs_pyoracle(nodes, pods, bound, prof)
    (pi, nom, victims), = s.preemptions
    assert s.node_names[nom] == "node-0" and [pods[v].name for v in victims] == ["a"]


@pytest.mark.parametrize("seed", [31, 32])
def test_volume_preemptors_vs_pyoracle(seed):
    """Preemptors with claims (zonal / local / plain PVs, one ReadWriteOncePod
    claim a higher-priority running pod holds): VolumeBinding / VolumeZone
    ordered after Fit filter the candidates, VolumeRestrictions' conflict
    leaves none."""
    nodes, pods, bound, prof = G.preemption_volume_case(seed=seed)
    nb = len(bound)
    s = _vs_pyoracle(nodes, pods, bound, prof)
    claimants = [pi for pi, _, _ in s.preemptions if pods[pi].claim_names()]
    assert len(claimants) >= 5
    assert pods[nb].claim_names() == ["rwop-0"] and nb not in {pi for pi, _, _ in s.preemptions}


def test_eval_skipping_and_eval_pod_with_claims():
    """The oracle's ksg_eval_skipping: no status word names a skipped plugin,
    every node ksg_eval passes still passes, and the record is restored; its
    ksg_eval_pod of a pod with claims (the volume program rebased) equals
    ksg_eval."""
    E = pkg("encoder")
    nodes, pods, bound, prof = G.preemption_volume_case(seed=31)
    enc = E.Encoder(nodes, pods, prof, bound_pods=[i for i, _ in bound])
    eng = _oracle_engine()
    eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    N, mask = len(nodes), PR.static_skip_mask()
    n_vol = 0
    for pi in range(len(bound), len(pods), 2):
        a, b, c = (native.CaptureBuffers(N) for _ in range(3))
        r0 = eng.eval(pi, a)
        eng.eval_skipping(pi, mask, b)
        fa, fb = np.asarray(a.fstatus[0]), np.asarray(b.fstatus[0])
        assert not any((mask >> ((int(w) & 0xFF) - 1)) & 1 for w in fb if w and w != 0xFFFFFFFF)
        assert np.all(fb[fa == 0] == 0)
        r1 = eng.eval(pi, c)
        assert (r0.selected, r0.n_feasible, r0.status) == (r1.selected, r1.n_feasible, r1.status)
        rec = enc.workload.pods[pi].copy()
        if int(rec["vol"]) < 0 or int(rec["node_set"]) >= 0:
            continue
        n_vol += 1
        lo, hi = int(rec["blob"]), int(rec["blob"]) + int(rec["blob_len"])
        for f in ("tol", "na_req", "na_pref", "img", "pts", "ipa", "commit", "blob", "ports", "vol"):
            if int(rec[f]) >= 0:
                rec[f] = int(rec[f]) - lo
        d = native.CaptureBuffers(N)
        r2 = eng.eval_pod(rec, enc.workload.prog[lo:hi], d)
        assert (r2.selected, r2.n_feasible, r2.status) == (r0.selected, r0.n_feasible, r0.status)
        np.testing.assert_array_equal(d.fstatus, a.fstatus)
    assert n_vol >= 5


def test_rwop_holder_refusal():
    """The one case refused: every holder of the preemptor's
    ReadWriteOncePod claim a potential victim on one node."""
    nodes, pods, bound, prof = _kat(100)
    st = m.Storage()
    pv = m.PersistentVolume("pv-r", claim_ref=("default", "r"))
    st.pvs[pv.name] = pv
    st.pvcs[("default", "r")] = m.PersistentVolumeClaim("r", "default", "pv-r", "", ("ReadWriteOncePod",),
                                                        {m.ANN_BIND_COMPLETED: "yes"})
    for p in pods:
        p.storage = st
    pods[0].volumes = [("v0", "persistentVolumeClaim", "r")]     # a (prio 1) on node-0
    pods[-1].volumes = [("v0", "persistentVolumeClaim", "r")]
    assert PR.status_code(1 + P.VOLUME_RESTRICTIONS) == PR.UNSCHEDULABLE
    with pytest.raises(NotImplementedError):
        _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    pods[0].priority = 10                                         # the holder outranks nobody: no candidate
    pods[-1].priority = 10
    s, placed, _ = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    assert placed == [-1] and not s.preemptions


def _topo_preemptors(s, pods):
    return [pi for pi, _, _ in s.preemptions
            if pods[pi].topology_spread_constraints or pods[pi].pod_anti_affinity_required
            or pods[pi].pod_affinity_required]


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_topology_preemption_framework_vs_pyoracle(seed):
    """Preemptors with DoNotSchedule spread constraints / required inter-pod
    terms, and victims carrying required anti-affinity: the C++ oracle's dry
    run (PreFilter state recomputed) against pyoracle's, annotation bytes
    included."""
    nodes, pods, bound, prof = G.preemption_topo_case(seed=seed)
    s, placed, ann = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert _topo_preemptors(s, pods), "no preemption by a topology-constrained pod"
    assert [r["selected_index"] for r in recs] == placed
    pre = [(pi - nb, s.node_names[n], [(pods[v].namespace, pods[v].name) for v in vs]) for pi, n, vs in s.preemptions]
    ref = [(k, r["first_attempt"]["nominated"], r["first_attempt"]["victims"])
           for k, r in enumerate(recs) if "first_attempt" in r]
    assert pre == ref
    assert ann == ora


def _port_preemptions(s, pods):
    return [pi for pi, _, _ in s.preemptions if pods[pi].host_ports()]


@pytest.mark.parametrize("seed", [31, 32, 33])
def test_host_port_preemption_framework_vs_pyoracle(seed):
    """Preemptors with host ports: the dry run re-runs
    NodePorts on the UsedPorts the removed / reprieved victims leave (C++
    oracle: set semantics, as upstream's HostPortInfo) against pyoracle's
    trial NodeInfo, annotation bytes included.  Parity vs Go unpinned."""
    nodes, pods, bound, prof = G.preemption_ports_case(seed=seed)
    s, placed, ann = _run_framework(_oracle_engine(), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert _port_preemptions(s, pods), "no preemption by a pod with host ports"
    assert [r["selected_index"] for r in recs] == placed
    pre = [(pi - nb, s.node_names[n], [(pods[v].namespace, pods[v].name) for v in vs]) for pi, n, vs in s.preemptions]
    ref = [(k, r["first_attempt"]["nominated"], r["first_attempt"]["victims"])
           for k, r in enumerate(recs) if "first_attempt" in r]
    assert pre == ref
    assert ann == ora


# ---- GPU: the dry run and the deletions on the device ------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("seed", [31, 32, 34])
def test_gpu_host_port_preemption_matches_pyoracle(built, seed):
    """The device's dry run with NodePorts (PrePorts: the preemptor's conflict
    ids tracked through the removals and reprieves) against pyoracle."""
    nodes, pods, bound, prof = G.preemption_ports_case(seed=seed, n_nodes=60, n_bound=260, n_queue=160)
    s, placed, ann = _run_framework(native.Engine(device=0), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert _port_preemptions(s, pods)
    assert [r["selected_index"] for r in recs] == placed
    assert ann == ora



@pytest.mark.gpu
@pytest.mark.parametrize("seed", [31, 32, 33])
def test_gpu_volume_preemptors_match_pyoracle(built, seed):
    """Preemptors with claims on the device: ksg_eval_skipping's node-static
    verdict (VolumeBinding / VolumeZone after Fit) against pyoracle."""
    nodes, pods, bound, prof = G.preemption_volume_case(seed=seed, n_nodes=60, n_bound=260, n_queue=160)
    s = _vs_pyoracle(nodes, pods, bound, prof, native.Engine(device=0))
    assert [pi for pi, _, _ in s.preemptions if pods[pi].claim_names()]


@pytest.mark.gpu
def test_gpu_static_filter_after_fit(built):
    nodes, pods, bound, prof = _kat(100)
    f = m.Pod(name="f", containers=[m.Container(image="pause", requests={m.CPU: 4000, m.MEMORY: GI})])
    f.priority, f.start_time, f.node_name = 0, 5, "node-2"
    pods.insert(5, f)
    bound.append((5, 2))
    names = [n for n, _ in prof.plugins]
    i, j = names.index("TaintToleration"), names.index("NodeResourcesFit")
    prof.plugins[i], prof.plugins[j] = prof.plugins[j], prof.plugins[i]
    s = _vs_pyoracle(nodes, pods, bound, prof, native.Engine(device=0))
    assert [s.node_names[n] for _, n, _ in s.preemptions] == ["node-0"]


@pytest.mark.gpu
def test_gpu_eval_skipping_equals_oracle(built):
    """ksg_eval_skipping on every pod of a volume case, equal to the oracle's
    twin and leaving the record as it was (a plain ksg_eval after it)."""
    E = pkg("encoder")
    nodes, pods, bound, prof = G.preemption_volume_case(seed=33)
    enc = E.Encoder(nodes, pods, prof, bound_pods={i for i, _ in bound})
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu, cpu = native.Engine(device=0), _oracle_engine()
    gpu.load(enc, pf)
    cpu.load(enc, pf)
    N = len(nodes)
    for pi in range(len(bound), len(pods), 3):
        a, b = native.CaptureBuffers(N), native.CaptureBuffers(N)
        ra = gpu.eval_skipping(pi, PR.static_skip_mask(), a)
        rb = cpu.eval_skipping(pi, PR.static_skip_mask(), b)
        assert (ra.selected, ra.n_feasible) == (rb.selected, rb.n_feasible)
        np.testing.assert_array_equal(a.fstatus, b.fstatus)
        a2, b2 = native.CaptureBuffers(N), native.CaptureBuffers(N)
        r2, r3 = gpu.eval(pi, a2), cpu.eval(pi, b2)
        assert (r2.selected, r2.n_feasible, r2.status) == (r3.selected, r3.n_feasible, r3.status)
        np.testing.assert_array_equal(a2.fstatus, b2.fstatus)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [7, 8, 9, 10])
def test_gpu_preemption_matches_pyoracle(built, seed):
    nodes, pods, bound, prof = G.preemption_case(seed=seed, n_nodes=60, n_bound=260, n_queue=160)
    s, placed, ann = _run_framework(native.Engine(device=0), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert s.preemptions
    assert [r["selected_index"] for r in recs] == placed
    assert ann == ora


@pytest.mark.gpu
def test_gpu_kat_and_run_queue(built):
    for a_start, node in ((100, "node-0"), (20, "node-1")):
        nodes, pods, bound, prof = _kat(a_start)
        s, placed, _ = _run_framework(native.Engine(device=0), nodes, pods, bound, prof)
        assert s.node_names[placed[0]] == node
    nodes, pods, bound, prof = G.preemption_case(seed=11, n_nodes=200, n_bound=900, n_queue=1500)
    nb = len(bound)
    s_gpu = F.DebuggableScheduler(nodes, pods, prof, engine=native.Engine(device=0), bound=bound)
    pl, _ = s_gpu.run_queue(nb, len(pods) - nb)
    s_cpu = F.DebuggableScheduler(nodes, pods, prof, engine=_oracle_engine(), bound=bound)
    pl2, _ = s_cpu.run_queue(nb, len(pods) - nb)
    np.testing.assert_array_equal(pl, pl2)
    assert s_gpu.preemptions == s_cpu.preemptions
    req_g = s_gpu.engine.read_state(3)
    req_c = s_cpu.engine.read_state(3)
    for a, b in zip(req_g, req_c):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_gpu_topology_preemption_matches_pyoracle(built, seed):
    """The device's topology dry run (ksg_preempt_prepass + ksg_preempt_topo:
    incremental domain counts) against pyoracle's recomputed PreFilter state."""
    nodes, pods, bound, prof = G.preemption_topo_case(seed=seed, n_nodes=60, n_bound=260, n_queue=160)
    s, placed, ann = _run_framework(native.Engine(device=0), nodes, pods, bound, prof)
    nb = len(bound)
    ora, recs = pyoracle_annotations(nodes, pods[nb:], prof, bound=[(pods[i], nodes[n].name) for i, n in bound])
    assert _topo_preemptors(s, pods)
    assert [r["selected_index"] for r in recs] == placed
    assert ann == ora


@pytest.mark.gpu
def test_gpu_topology_preemption_victims_match_cpp_oracle(built):
    """Victim flags of every candidate of every preemption: device vs C++ oracle."""
    nodes, pods, bound, prof = G.preemption_topo_case(seed=25, n_nodes=80, n_bound=400, n_queue=200)
    nb = len(bound)
    s_gpu = F.DebuggableScheduler(nodes, pods, prof, engine=native.Engine(device=0), bound=bound)
    s_cpu = F.DebuggableScheduler(nodes, pods, prof, engine=_oracle_engine(), bound=bound)
    for i in range(nb, len(pods)):
        assert s_gpu.schedule_one(i) == s_cpu.schedule_one(i), i
    assert s_gpu.preemptions == s_cpu.preemptions and _topo_preemptors(s_gpu, pods)


def _many_anti_templates(n_templates: int):
    """Four nodes, one low-priority running pod per existing anti-affinity
    template (selector k<i>=x, hostname), and a high-priority preemptor whose
    labels match every template: its InterPodAffinity program lists
    n_templates existing-pod anti-affinity templates."""
    nodes = [m.Node(name=f"node-{i}", labels={m.LABEL_HOSTNAME: f"node-{i}"},
                    allocatable={m.CPU: 4000, m.MEMORY: 16 * GI, m.PODS: 110}) for i in range(4)]
    pods, bound = [], []
    for i in range(n_templates):
        p = m.Pod(name=f"run-{i}", containers=[m.Container(image="pause", requests={m.CPU: 200, m.MEMORY: GI})])
        p.priority, p.node_name = 1, f"node-{i % 4}"
        p.pod_anti_affinity_required = [m.PodAffinityTerm(m.LabelSelector(match_labels=((f"k{i}", "x"),)),
                                                          m.LABEL_HOSTNAME)]
        pods.append(p)
        bound.append((i, i % 4))
    pre = m.Pod(name="preemptor", labels={f"k{i}": "x" for i in range(n_templates)},
                containers=[m.Container(image="pause", requests={m.CPU: 3000, m.MEMORY: GI})])
    pre.priority = 10
    pods.append(pre)
    return nodes, pods, bound, P.default_profile()


@pytest.mark.gpu
@pytest.mark.parametrize("n_templates", [16, 17])
def test_gpu_preemption_refuses_too_many_anti_templates(built, n_templates):
    """The topology dry run holds 16 existing anti-affinity templates per
    preemptor; 17 are refused on the host before any launch, 16
    run and agree with the C++ oracle."""
    E = pkg("encoder")
    nodes, pods, bound, prof = _many_anti_templates(n_templates)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu, cpu = native.Engine(device=0), _oracle_engine()
    for eng in (gpu, cpu):
        eng.load(enc, pf)
        for pi, ni in bound:
            eng.commit(pi, ni)
    pre = len(pods) - 1
    cand = [0, 1, 2, 3]
    lists = [[q for q, n in bound if n == c] for c in cand]
    off = np.concatenate([[0], np.cumsum([len(v) for v in lists])]).astype(np.int32)
    vic = np.array([q for v in lists for q in v], np.int32)
    if n_templates > 16:
        with pytest.raises(native.KschedError, match="anti-affinity templates"):
            gpu.preempt_victims(pre, cand, off, vic)
        return
    fg, vg = gpu.preempt_victims(pre, cand, off, vic)
    fc, vc = cpu.preempt_victims(pre, cand, off, vic)
    np.testing.assert_array_equal(fg, fc)
    np.testing.assert_array_equal(vg, vc)
