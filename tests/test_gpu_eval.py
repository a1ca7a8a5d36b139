"""The per-cycle path (ksg_eval): one pod's PreFilter ..
NormalizeScore on the chip-wide kernels with persistent buffers, as the Go
shim calls it once per scheduling cycle, against the C++ oracle's ksg_eval
(kso_eval) pod by pod: result, every node's status word, the score plugins'
raw / normalised rows and the totals; each pod is then assumed on both (the
host-driven eval -> commit loop).  Topology pods take the chip-wide topology
kernel's evaluate-only capture form (path 6) into the same pinned block."""
import os

import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
native = pkg("native")
m = pkg("model")

pytestmark = pytest.mark.gpu

CASES = {
    "c2-1000x120": lambda: G.config2(n_nodes=1000, n_pods=120, seed=3),
    "c2-tight": lambda: G.config2(n_nodes=7, n_pods=60, seed=11),
    "c2-most": lambda: (lambda n, p, _: (n, p, P.config2_profile(strategy=P.MOST_ALLOCATED)))(
        *G.config2(n_nodes=300, n_pods=80, seed=12)),
    "c1-100x150": lambda: G.config1(n_nodes=100, n_pods=150),
    "c5-small": lambda: G.config5(n_nodes=400, n_pods=60, n_images=200, taint_vocab=128, taints_per_node=16,
                                  images_per_node=20),
    "c3-60x80": lambda: G.config3(n_nodes=60, n_pods=80, apps=12, zones=4),
    "c3-15000x40": lambda: G.config3(n_nodes=15000, n_pods=40, apps=30, zones=16),
    "readme-kat2": G.readme_kat2,
    # taint vocabulary of 8,192: toleration bitmaps of 512 words (programs too
    # long for the kernel arguments) and effects too many for the LDS copy
    "c5-vocab8k": lambda: G.config5(n_nodes=300, n_pods=40, n_images=100, taint_vocab=8192, taints_per_node=12,
                                    images_per_node=10),
    "c1-images": lambda: G.config1(n_nodes=700, n_pods=60, seed=5),
}
CASES.update({f"zoo-{s}": (lambda s=s: __import__("zoo").zoo(s, n_pods=60)) for s in range(4)})
CASES.update({f"zoo-{k}-{s}": (lambda s=s, k=k: __import__("zoo").zoo_args(s, k, n_pods=60))
              for k in ("rtcr", "pts-list") for s in (0, 2)})


@pytest.fixture(scope="module")
def gpu(built):
    return native.Engine(device=0)


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


def _score_rows(pf):
    return [p for p in range(native.NPLUGINS) if (pf["score_mask"] >> p) & 1]


@pytest.mark.parametrize("name", sorted(CASES))
def test_eval_cycle_matches_oracle(gpu, oracle, name):
    _check_cycles(gpu, oracle, name, *CASES[name]())


@pytest.mark.parametrize("kn", [2, 4])
@pytest.mark.parametrize("name", ["c2-1000x120", "c5-small", "zoo-1"])
def test_eval_cycle_nodes_per_lane(oracle, monkeypatch, kn, name):
    """KN = 2 and 4 nodes per lane (the per-cycle kernel's form above ~98 k
    nodes, forced here by KSG_CYCLE_KN) equal the oracle as KN = 1 does."""
    monkeypatch.setenv("KSG_CYCLE_KN", str(kn))
    eng = native.Engine(device=0)
    try:
        _check_cycles(eng, oracle, name, *CASES[name]())
    finally:
        eng.close()


@pytest.mark.parametrize("name", ["c2-1000x120", "c1-100x150", "c5-small", "c5-vocab8k", "zoo-0", "zoo-3",
                                  "readme-kat2"])
def test_eval_cycle_launch_matches_oracle(oracle, monkeypatch, name):
    """One ksg_eval_cycle launch per cycle (KSG_CYCLE_SERVER=0; the persistent
    server, which test_eval_cycle_matches_oracle runs, is the default since
    round 6) equals the oracle pod by pod, deferred assumes included."""
    monkeypatch.setenv("KSG_CYCLE_SERVER", "0")
    eng = native.Engine(device=0)
    try:
        _check_cycles(eng, oracle, name, *CASES[name]())
    finally:
        eng.close()


def test_eval_cycle_server_across_reloads(oracle, monkeypatch):
    """One context, two workloads, the persistent server running for both: a
    reload stops the server and reallocates its relay block, and the next
    server must not take the zeroed relay for a call (round 6 fix)."""
    monkeypatch.setenv("KSG_CYCLE_SERVER", "1")
    eng = native.Engine(device=0)
    try:
        for name in ("c2-1000x120", "c1-100x150", "zoo-1"):
            _check_cycles(eng, oracle, name, *CASES[name]())
    finally:
        eng.close()


def test_eval_cycle_server_interleaved_with_queue_runs(oracle, monkeypatch):
    """Calls that need the stream (a queue run, a non-deferrable assume, a
    reload) stop the server and the next evaluation starts it again, reading
    the node state those calls left."""
    monkeypatch.setenv("KSG_CYCLE_SERVER", "1")
    nodes, pods, prof = G.config2(n_nodes=700, n_pods=90, seed=21)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng = native.Engine(device=0)
    try:
        eng.load(enc, pf)
        oracle.load(enc, pf)
        for lo, hi, how in ((0, 30, "eval"), (30, 50, "queue"), (50, 70, "eval"), (70, 75, "queue"), (75, 90, "eval")):
            if how == "queue":
                pg, _ = eng.run_queue(lo, hi - lo, results=False)
                po, _ = oracle.run_queue(lo, hi - lo, results=False)
                np.testing.assert_array_equal(pg, po)
                continue
            for i in range(lo, hi):
                rg, ro = eng.eval(i), oracle.eval(i)
                assert (rg.selected, rg.n_feasible, rg.status) == (ro.selected, ro.n_feasible, ro.status), i
                if rg.selected >= 0:
                    eng.commit(i, rg.selected)
                    oracle.commit(i, ro.selected)
        R = len(enc.cluster.res_names)
        for a, b in zip(eng.read_state(R), oracle.read_state(R)):
            np.testing.assert_array_equal(a, b)
    finally:
        eng.close()


def _check_cycles(gpu, oracle, name, nodes, pods, prof):
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    N = len(nodes)
    rows = _score_rows(pf)
    fast = 0
    for i in range(len(pods)):
        cg, co = native.CaptureBuffers(N, 1), native.CaptureBuffers(N, 1)
        rg, ro = gpu.eval(i, cg), oracle.eval(i, co)
        fast += gpu.last_run_info()[0] in (5, 6)
        assert (rg.selected, rg.n_feasible, rg.status, rg.score_skip) == \
            (ro.selected, ro.n_feasible, ro.status, ro.score_skip), (name, i)
        np.testing.assert_array_equal(cg.fstatus, co.fstatus, err_msg=f"{name} pod {i} status words")
        if ro.status & native.ST_SCORED:
            feas = co.fstatus[0] == 0
            for pid in rows:
                if (ro.score_skip >> pid) & 1:
                    continue
                np.testing.assert_array_equal(cg.raw[0, pid][feas], co.raw[0, pid][feas], err_msg=f"{name} {i} raw")
                np.testing.assert_array_equal(cg.norm[0, pid][feas], co.norm[0, pid][feas], err_msg=f"{name} {i}")
            np.testing.assert_array_equal(cg.total[0][feas], co.total[0][feas], err_msg=f"{name} pod {i} total")
        if rg.selected >= 0:
            gpu.commit(i, rg.selected)
            oracle.commit(i, ro.selected)
    R = len(enc.cluster.res_names)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    if name.startswith(("c2", "c1", "c5", "readme", "c3")):
        assert fast == len(pods), f"{name}: {fast} of {len(pods)} cycles on the per-cycle paths"


def test_eval_fast_equals_queue_kernel_capture(gpu, built):
    """The chip-wide per-cycle capture equals the single-workgroup queue
    kernel's (KSG_EVAL_FAST=0) on every row the profile scores, infeasible
    nodes included."""
    old = os.environ.get("KSG_EVAL_FAST")
    os.environ["KSG_EVAL_FAST"] = "0"
    try:
        slow = native.Engine(device=0)
    finally:
        if old is None:
            del os.environ["KSG_EVAL_FAST"]
        else:
            os.environ["KSG_EVAL_FAST"] = old
    nodes, pods, prof = G.config2(n_nodes=2000, n_pods=40, seed=8)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    slow.load(enc, pf)
    rows = _score_rows(pf)
    for i in range(len(pods)):
        a, b = native.CaptureBuffers(len(nodes), 1), native.CaptureBuffers(len(nodes), 1)
        ra, rb = gpu.eval(i, a), slow.eval(i, b)
        assert gpu.last_run_info()[0] == 5 and slow.last_run_info()[0] == 1
        assert (ra.selected, ra.n_feasible, ra.status, ra.score_skip) == (rb.selected, rb.n_feasible, rb.status,
                                                                           rb.score_skip)
        np.testing.assert_array_equal(a.fstatus, b.fstatus)
        np.testing.assert_array_equal(a.raw[:, rows], b.raw[:, rows])
        np.testing.assert_array_equal(a.norm[:, rows], b.norm[:, rows])
        if ra.selected >= 0:
            gpu.commit(i, ra.selected)
            slow.commit(i, rb.selected)


def test_eval_without_capture_and_eval_pod(gpu, oracle):
    """No capture buffers (placement only), and ksg_eval_pod of an encoded pod
    outside the workload, on the per-cycle path."""
    nodes, pods, prof = G.config2(n_nodes=500, n_pods=30, seed=4)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    for i in range(len(pods)):
        rg, ro = gpu.eval(i), oracle.eval(i)
        assert (rg.selected, rg.n_feasible, rg.status) == (ro.selected, ro.n_feasible, ro.status)
        rec = enc.workload.pods[i].copy()
        lo, hi = int(rec["blob"]), int(rec["blob"]) + int(rec["blob_len"])
        for f in ("tol", "na_req", "na_pref", "img", "node_set", "pts", "ipa", "commit", "blob"):
            if int(rec[f]) >= 0:
                rec[f] = int(rec[f]) - lo
        rp = gpu.eval_pod(rec, enc.workload.prog[lo:hi])
        assert (rp.selected, rp.n_feasible, rp.status) == (ro.selected, ro.n_feasible, ro.status)
        if rg.selected >= 0:
            gpu.commit(i, rg.selected)
            oracle.commit(i, ro.selected)


def test_cycles_from_an_empty_snapshot(built):
    """The Go shim's life cycle from an empty pod set (bench.py per_cycle):
    nodes only at load, then add_pod -> sync -> eval -> statuses -> assume per
    pod; placements equal one device queue over the same pods."""
    S = pkg("snapshot")
    nodes, pods, prof = G.config2(n_nodes=400, n_pods=150, seed=6)
    snap = S.Snapshot(prof, nodes)
    eng = native.Engine(device=0)
    snap.load(eng)
    cap = native.CaptureBuffers(len(nodes), 1)
    placed = []
    for p in pods:
        idx = snap.add_pod(p)
        snap.sync(eng)
        r = eng.eval(idx, cap)
        codes, msg, texts = snap.statuses(idx, cap.fstatus[0])
        assert ((codes != 0) == (msg >= 0)).all()
        if r.selected >= 0:
            snap.assume(eng, idx, r.selected)
        placed.append(r.selected)
    enc = E.Encoder(nodes, pods, prof)
    q = native.Engine(device=0)
    q.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    want, _ = q.run_queue(0, len(pods), results=False)
    np.testing.assert_array_equal(np.array(placed, np.int32), want)


def test_eval_view_equals_eval_with_capture(gpu, built):
    """ksg_eval_view leaves the rows in library memory: the same status words,
    raw / normalised rows and totals as ksg_eval with capture buffers, on the
    per-cycle path and (topology pods) its chip-wide topology form.  The
    node-local per-cycle kernel stores no normalised rows and no totals
    (round 6): the view's TaintToleration / NodeAffinity rows are derived from
    the raw rows and the maxima (native.derive_norm), as the Go shim derives
    them, and must equal the capture's (which test_eval_cycle_matches_oracle
    compares with the oracle's)."""
    import zoo
    for nodes, pods, prof in (G.config2(n_nodes=1500, n_pods=30, seed=3), zoo.zoo(2, n_pods=40)):
        _view_equals_capture(gpu, nodes, pods, prof)


def test_eval_view_row_widths(built):
    """The per-cycle rows are one byte wide while every raw score fits in
    [0, 255], two bytes for a pod whose preferred node-affinity weights sum
    past it; both equal ksg_eval's capture.  (Its own engine, closed at the
    end: no server of it outlives the test.)"""
    nodes, pods, prof = G.config2(n_nodes=1500, n_pods=30, seed=3)
    for p in pods[::3]:
        p.node_affinity_preferred = [m.PreferredSchedulingTerm(100, m.NodeSelectorTerm(match_expressions=(
            m.Requirement("pool", m.IN, (pool,)),))) for pool in G.POOLS[:3]]
    eng = native.Engine(device=0)
    try:
        widths = _view_equals_capture(eng, nodes, pods, prof)
    finally:
        eng.close()
    assert widths == {1, 2}


def _view_equals_capture(gpu, nodes, pods, prof):
    widths = set()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    rows = _score_rows(pf)
    for i in range(len(pods)):
        cap = native.CaptureBuffers(len(nodes), 1)
        ra = gpu.eval(i, cap)
        rv, v = gpu.eval_view(i)
        widths.add(v["elem_bytes"])
        assert (ra.selected, ra.n_feasible, ra.status, ra.score_skip) == (rv.selected, rv.n_feasible, rv.status,
                                                                           rv.score_skip)
        np.testing.assert_array_equal(cap.fstatus[0], v["fstatus"])
        assert sorted(v["raw"]) == sorted(rows)
        for p in rows:
            np.testing.assert_array_equal(cap.raw[0, p], v["raw"][p])
            np.testing.assert_array_equal(cap.norm[0, p], v["norm"][p])
        if v["total"] is not None:   # (the node-local per-cycle kernel leaves the totals out)
            np.testing.assert_array_equal(cap.total[0], v["total"])
        else:
            assert gpu.last_run_info()[0] == 5
        if ra.selected >= 0:
            gpu.commit(i, ra.selected)
    return widths


def _engine_with(env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return native.Engine(device=0)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_deferred_assume_reaches_every_reader(built):
    """ksg_commit after a per-cycle evaluation is applied by the next
    per-cycle kernel (or launched first by any other reader of the node
    state): evaluations, read_state, run_queue, uncommit and reset_state see
    the same state as with every assume launched at once (KSG_DEFER_COMMIT=0)."""
    nodes, pods, prof = G.config2(n_nodes=600, n_pods=60, seed=9)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = native.Engine(device=0)
    b = _engine_with({"KSG_DEFER_COMMIT": "0"})
    a.load(enc, pf)
    b.load(enc, pf)
    R = len(enc.cluster.res_names)

    def same_state():
        for x, y in zip(a.read_state(R), b.read_state(R)):
            np.testing.assert_array_equal(x, y)

    for i in range(40):
        ra, rb = a.eval(i), b.eval(i)
        assert a.last_run_info()[0] == 5
        assert (ra.selected, ra.n_feasible, ra.status) == (rb.selected, rb.n_feasible, rb.status), i
        if ra.selected < 0:
            continue
        a.commit(i, ra.selected)
        b.commit(i, rb.selected)
        k = i % 6
        if k == 1:
            same_state()
        elif k == 2:   # the queue kernels read the state after the pending assume
            pa, _ = a.run_queue(50, 2, results=False)
            pb, _ = b.run_queue(50, 2, results=False)
            np.testing.assert_array_equal(pa, pb)
        elif k == 3:   # forget the pod just assumed (pending on a)
            a.uncommit(i, ra.selected)
            b.uncommit(i, rb.selected)
            same_state()
        elif k == 4:   # two assumes in a row: the first is launched, the second deferred
            a.commit(i, ra.selected)
            b.commit(i, rb.selected)
    same_state()
    a.reset_state()   # a pending assume is dropped with the rest
    b.reset_state()
    same_state()


def test_commit_batch_equals_sequential_commits(built):
    """ksg_commit_batch (one launch, atomic additions; the snapshot's replay of
    its bindings) leaves the node state, selector counts and template tables
    exactly as one ksg_commit per pod does: later evaluations agree, topology
    pods included."""
    import zoo
    nodes, pods, prof = zoo.zoo(1, n_nodes=300, n_pods=120)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    a = native.Engine(device=0)
    b = _engine_with({"KSG_DEFER_COMMIT": "0"})
    a.load(enc, pf)
    b.load(enc, pf)
    rng = np.random.default_rng(5)
    bp = np.arange(0, 80, dtype=np.int32)
    bn = rng.integers(0, len(nodes), size=len(bp)).astype(np.int32)
    bn[:10] = 7   # several pods on one node: lanes sharing a node
    a.commit_batch(bp, bn)
    for q, n in zip(bp, bn):
        b.commit(int(q), int(n))
    R = len(enc.cluster.res_names)
    for x, y in zip(a.read_state(R), b.read_state(R)):
        np.testing.assert_array_equal(x, y)
    for i in range(80, len(pods)):   # selector counts and template tables: later pods see the same state
        ca, cb = native.CaptureBuffers(len(nodes), 1), native.CaptureBuffers(len(nodes), 1)
        ra, rb = a.eval(i, ca), b.eval(i, cb)
        assert (ra.selected, ra.n_feasible, ra.status) == (rb.selected, rb.n_feasible, rb.status), i
        np.testing.assert_array_equal(ca.fstatus, cb.fstatus)
        np.testing.assert_array_equal(ca.total, cb.total)


def test_topology_cycles_with_tables_across_invalidations(gpu, oracle):
    """The per-cycle topology tables (built once, kept exact by ksg_commit /
    ksg_uncommit, rebuilt after anything else moved the counts): evaluate +
    assume, uncommit a few assumes, a queue run, a reset, more cycles; every
    cycle equal to the oracle's, the node state too."""
    nodes, pods, prof = G.config3(n_nodes=400, n_pods=160, apps=10, zones=4)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    N, R = len(nodes), len(enc.cluster.res_names)

    def cycles(lo, hi, placed):
        for i in range(lo, hi):
            cg, co = native.CaptureBuffers(N, 1), native.CaptureBuffers(N, 1)
            rg, ro = gpu.eval(i, cg), oracle.eval(i, co)
            assert gpu.last_run_info()[0] == 6
            assert (rg.selected, rg.n_feasible, rg.status) == (ro.selected, ro.n_feasible, ro.status), i
            np.testing.assert_array_equal(cg.fstatus, co.fstatus, err_msg=f"pod {i}")
            np.testing.assert_array_equal(cg.total, co.total, err_msg=f"pod {i}")
            if rg.selected >= 0:
                gpu.commit(i, rg.selected)
                oracle.commit(i, ro.selected)
                placed.append((i, rg.selected))

    placed = []
    cycles(0, 40, placed)
    for i, n in placed[::3][:6]:   # victims' deletions (ksg_uncommit: the tables follow)
        gpu.uncommit(i, n)
        oracle.uncommit(i, n)
    cycles(40, 70, placed)
    pl_g, _ = gpu.run_queue(70, 30)   # a queue run moves the counts: the tables are rebuilt
    pl_o, _ = oracle.run_queue(70, 30)
    np.testing.assert_array_equal(pl_g, pl_o)
    cycles(100, 130, placed)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    gpu.reset_state()
    oracle.reset_state()
    cycles(130, 160, [])
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
