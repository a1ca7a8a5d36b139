"""Scenario driver and requeue semantics (KEP-140 /
KEP-184).  The scenarios are small and worked by hand: which pods bind at
which MajorStep, which unschedulable pods a cluster event moves back to the
active queue (and which it must leave alone), preemption inside a scenario,
and the KEP-184 what-if fan-out over ranks (gloo, world size 2).  The engine
is the C++ oracle on CPU; the GPU test runs the same scenarios through
libksched.so and requires byte-identical results."""
import json
import os
import socket

import pytest

from conftest import pkg

I = pkg("ingest")
m = pkg("model")
P = pkg("profile")
S = pkg("scenario")
A = pkg("annotations")
native = pkg("native")

GI = 1024 ** 3


def _node(name, cpu=4000, taint=None):
    n = m.Node(name=name, labels={m.LABEL_HOSTNAME: name},
               allocatable={m.CPU: cpu, m.MEMORY: 16 * GI, m.EPHEMERAL: 100 * GI, m.PODS: 110})
    if taint:
        n.taints = [m.Taint(taint, "x", m.NO_SCHEDULE)]
    return I.node_to_k8s(n)


def _pod(name, cpu, prio=0, tolerate=None):
    p = m.Pod(name=name, containers=[m.Container(image="pause", requests={m.CPU: cpu, m.MEMORY: GI})])
    p.priority = prio
    if tolerate:
        p.tolerations = [m.Toleration(tolerate, "Exists", "", m.NO_SCHEDULE)]
    return I.pod_to_k8s(p)


def _create(step, obj):
    return {"step": step, "createOperation": {"object": obj}}


def _delete(step, kind, name):
    return {"step": step, "deleteOperation": {"typeMeta": {"kind": kind},
                                              "objectMeta": {"name": name, "namespace": "default"}}}


def scenario_basic():
    """step 0: node-a (4 cores), p1 (3) and p2 (3): p1 binds, p2 fails (Fit).
    step 1: node-b (tainted) arrives: the Node/Add event returns p2 to the
    active queue, and p2 fails again (Fit on node-a, TaintToleration on
    node-b); t1 (tolerating nothing) fails the same way.
    step 2: p1 is deleted: p2 (Fit-rejected) returns and binds on node-a;
    t1 was rejected by Fit too, so it returns and fails again.
    step 3: node-c arrives: t1 binds there.  step 4: done."""
    return {"spec": {"operations": [
        _create(0, _node("node-a")), _create(0, _pod("p1", 3000)), _create(0, _pod("p2", 3000)),
        _create(1, _node("node-b", taint="dedicated")), _create(1, _pod("t1", 2000)),
        _delete(2, "Pod", "p1"),
        _create(3, _node("node-c")),
        {"step": 4, "doneOperation": {}},
    ]}}


def scenario_events():
    return {"spec": {"operations": [
        _create(0, _node("node-a", taint="dedicated")), _create(0, _pod("w", 1000, tolerate="dedicated")),
        _create(0, _pod("x", 1000)), _create(0, _pod("f", 4000, tolerate="dedicated")),
        _delete(1, "Pod", "w"),
        _create(2, _node("node-b")),
    ]}}


def scenario_preemption():
    return {"spec": {"operations": [
        _create(0, _node("node-a")), _create(0, _pod("low", 3000, prio=1)),
        _create(1, _pod("high", 3000, prio=100)),
        {"step": 2, "doneOperation": {}},
    ]}}


def _oracle():
    import binding
    return binding.Oracle(1)


def test_basic_scenario_steps_requeue_and_history():
    ops = S.load_scenario(json.dumps(scenario_basic()))
    res = S.ScenarioRunner(P.default_profile(), _oracle).run(ops)
    assert res["phase"] == "Succeeded"
    pods = res["pods"]
    assert set(pods) == {"default/p2", "default/t1"}            # p1 deleted at step 2
    assert pods["default/p2"]["nodeName"] == "node-a" and pods["default/p2"]["attempts"] == 3
    assert pods["default/t1"]["nodeName"] == "node-c" and pods["default/t1"]["attempts"] == 3
    sched = {(int(k), e["podScheduled"]["pod"]["name"]): e["podScheduled"]["nodeName"]
             for k, evs in res["timeline"].items() for e in evs if "podScheduled" in e}
    assert sched == {(0, "p1"): "node-a", (2, "p2"): "node-a", (3, "t1"): "node-c"}
    # every attempt is in result-history, the last one is the pod's current result
    hist = json.loads(pods["default/t1"]["annotations"][A.RESULT_HISTORY])
    assert len(hist) == 3
    assert [h[A.SELECTED_NODE] for h in hist] == ["", "", "node-c"]
    flt = json.loads(hist[0][A.FILTER])
    assert flt["node-a"]["NodeResourcesFit"] == "Insufficient cpu"
    assert flt["node-b"]["TaintToleration"].startswith("node(s) had untolerated taint")
    # minor steps advance with every operation, the scheduler's included
    steps0 = [e["step"]["minor"] for e in res["timeline"]["0"]]
    assert steps0 == list(range(len(steps0)))


def test_event_only_wakes_registered_plugins():
    """step 0: node-a (4 cores, tainted); w (1 core, tolerates) binds there;
    x (no toleration) fails on TaintToleration only; f (4 cores, tolerates)
    fails on NodeResourcesFit.  step 1: w is deleted: the Pod/Delete event
    returns f (Fit registers it) and f binds; x stays unschedulable
    (TaintToleration does not register Pod/Delete).  step 2: node-b arrives:
    the Node/Add event returns x, which binds on node-b."""
    res = S.ScenarioRunner(P.default_profile(), _oracle).run(S.load_scenario(scenario_events()))
    assert res["phase"] == "Paused"
    x, f = res["pods"]["default/x"], res["pods"]["default/f"]
    assert (x["nodeName"], x["attempts"]) == ("node-b", 2)
    assert (f["nodeName"], f["attempts"]) == ("node-a", 2)
    sched = {e["podScheduled"]["pod"]["name"]: int(k) for k, evs in res["timeline"].items() for e in evs
             if "podScheduled" in e}
    assert sched == {"w": 0, "f": 1, "x": 2}


def test_preemption_inside_a_scenario():
    res = S.ScenarioRunner(P.default_profile(), _oracle).run(S.load_scenario(scenario_preemption()))
    assert set(res["pods"]) == {"default/high"}
    assert res["pods"]["default/high"]["nodeName"] == "node-a"
    evs = res["timeline"]["1"]
    dels = [e for e in evs if "delete" in e]
    assert dels and dels[0]["delete"]["preemptedBy"]["name"] == "high"
    assert dels[0]["delete"]["operation"]["objectMeta"]["name"] == "low"


def test_patch_is_refused():
    with pytest.raises(NotImplementedError):
        S.load_scenario({"spec": {"operations": [{"step": 0, "patchOperation": {"patch": "{}"}}]}})


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _profiles():
    return [P.default_profile(), P.config2_profile(), P.config2_profile(strategy=P.MOST_ALLOCATED)]


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = S.simulate(scenario_basic(), _profiles(), _oracle, rank=rank, world=world)
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(out, f, sort_keys=True)
    dist.barrier()
    dist.destroy_process_group()


def test_simulate_what_ifs_gloo_two_ranks(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    want = json.dumps(S.simulate(scenario_basic(), _profiles(), _oracle), sort_keys=True)
    for r in range(2):
        assert open(tmp_path / f"r{r}.json").read() == want


@pytest.mark.gpu
def test_gpu_scenarios_match_oracle(built):
    for doc in (scenario_basic(), scenario_events(), scenario_preemption()):
        ops = S.load_scenario(doc)
        a = S.ScenarioRunner(P.default_profile(), lambda: native.Engine(device=0)).run(ops)
        b = S.ScenarioRunner(P.default_profile(), _oracle).run(ops)
        assert json.dumps(a, sort_keys=True) == json.dumps(b, sort_keys=True)
