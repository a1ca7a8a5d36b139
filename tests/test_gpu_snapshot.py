"""GPU runs through the native snapshot encoder (snapshot.Snapshot ->
ksg_snapshot_load / ksg_snapshot_sync): placements and results identical to
the oracle run on the Python encoder's arrays; ksg_eval_pod (an encoded pod
outside the workload) equal to ksg_eval of the same pod; the per-cycle path
(add -> sync -> eval -> assume) equal to one ksg_run_queue."""
import numpy as np
import pytest

from conftest import pkg

E = pkg("encoder")
G = pkg("generator")
S = pkg("snapshot")
native = pkg("native")

import zoo  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


CASES = [("c2", lambda: G.config2(n_nodes=500, n_pods=600)),
         ("c3", lambda: G.config3(n_nodes=300, n_pods=500)),
         ("c1", lambda: G.config1(n_nodes=100, n_pods=300))] + \
        [(f"zoo-{s}", (lambda s=s: zoo.zoo(s))) for s in range(3)] + \
        [(f"zoo-volumes-{s}", (lambda s=s: zoo.zoo_volumes(s))) for s in range(3)]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_snapshot_load_queue(built, oracle, name, make):
    nodes, pods, prof = make()
    snap = S.Snapshot(prof, nodes, pods)
    gpu = native.Engine(device=0)
    snap.load(gpu)
    pl, res = gpu.run_queue(0, len(pods))
    enc = E.Encoder(nodes, pods, prof)
    oracle.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    want, wres = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl, want)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(res[f], wres[f], err_msg=f)


def test_eval_pod_equals_eval(built):
    nodes, pods, prof = zoo.zoo(5)
    enc = E.Encoder(nodes, pods, prof)
    gpu = native.Engine(device=0)
    gpu.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    N = len(nodes)
    for pi in range(0, len(pods), 7):
        rec = enc.workload.pods[pi].copy()
        lo, hi = int(rec["blob"]), int(rec["blob"]) + int(rec["blob_len"])
        ns = int(rec["node_set"])
        if ns >= 0:
            continue   # the node set lives outside the blob
        for f in ("tol", "na_req", "na_pref", "img", "pts", "ipa", "commit", "blob"):
            if rec[f] >= 0:
                rec[f] -= lo
        a, b = native.CaptureBuffers(N), native.CaptureBuffers(N)
        r1 = gpu.eval(pi, a)
        r2 = gpu.eval_pod(rec, enc.workload.prog[lo:hi], b)
        assert (r1.selected, r1.n_feasible, r1.status, r1.score_skip) == \
               (r2.selected, r2.n_feasible, r2.status, r2.score_skip)
        np.testing.assert_array_equal(a.fstatus, b.fstatus)
        np.testing.assert_array_equal(a.raw, b.raw)
        np.testing.assert_array_equal(a.norm, b.norm)
        if r1.selected >= 0:
            gpu.commit(pi, r1.selected)


@pytest.mark.parametrize("name,make", CASES[:2], ids=[c[0] for c in CASES[:2]])
def test_per_cycle_sync_path(built, name, make):
    """The Go shim's loop: nodes loaded once, then per pod add -> sync
    (append or reload) -> eval -> assume; equal to one device queue."""
    nodes, pods, prof = make()
    pods = pods[:200]
    full = S.Snapshot(prof, nodes, pods)
    g1 = native.Engine(device=0)
    full.load(g1)
    want, _ = g1.run_queue(0, len(pods))
    snap = S.Snapshot(prof, nodes, pods[:1])
    g2 = native.Engine(device=0)
    snap.load(g2)
    got, appended = [], 0
    for j, p in enumerate(pods):
        if j > 0:
            snap.add_pod(p)
            appended += snap.sync(g2)
        r = g2.eval(j)
        got.append(r.selected)
        if r.selected >= 0:
            snap.assume(g2, j, r.selected)
    np.testing.assert_array_equal(np.array(got, np.int32), want)
    assert appended > 0


def test_eval_then_commit_topology(built, oracle):
    """ksg_eval must not assume (regression: without capture a topology pod
    took the chip-wide path, which assumes every pod it places, so an
    eval + commit counted the pod twice)."""
    nodes, pods, prof = G.config3(n_nodes=300, n_pods=120)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu = native.Engine(device=0)
    gpu.load(enc, pf)
    got = []
    for j in range(len(pods)):
        r = gpu.eval(j)
        got.append(r.selected)
        if r.selected >= 0:
            gpu.commit(j, r.selected)
    oracle.load(enc, pf)
    want, _ = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(np.array(got, np.int32), want)


def test_per_cycle_sync_path_volumes(built):
    """The per-cycle loop with claims: a pod with claims makes the sync
    re-encode (shared claims and storage objects are read from the whole
    snapshot); placements equal one device queue of the same snapshot."""
    nodes, pods, prof = zoo.zoo_volumes(1)
    full = S.Snapshot(prof, nodes, pods)
    g1 = native.Engine(device=0)
    full.load(g1)
    want, _ = g1.run_queue(0, len(pods))
    snap = S.Snapshot(prof, nodes, pods[:1])
    g2 = native.Engine(device=0)
    snap.load(g2)
    got = []
    for j, p in enumerate(pods):
        if j > 0:
            snap.add_pod(p)
            snap.sync(g2)
        r = g2.eval(j)
        got.append(r.selected)
        if r.selected >= 0:
            snap.assume(g2, j, r.selected)
    np.testing.assert_array_equal(np.array(got, np.int32), want)
