"""GPU parity: libksched.so (HIP, gfx950) against the CPU oracle, bit-exact.

Every test here runs through the C ABI on cuda:0 and compares with the C++
oracle (oracle/oracle.cpp) on the same encoded inputs: placements, per-node
filter status words, raw and normalised scores and totals of every scored pod,
node state after the queue, and the annotation bytes the wrapped plugins
would write."""
import numpy as np
import pytest

from conftest import pkg
from helpers import compare_engine_runs, pyoracle_annotations, scheduler_annotations

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(built):
    return native.Engine(device=0)


def _engine_with_batch_mode(mode, **env):
    """Engine whose batched path runs phase-2 variant `mode`; `env` sets further
    KSG_* knobs (e.g. KSG_SLOT_BLOCK).  All are read at ksg_open."""
    import os
    env = {"KSG_BATCH_MODE": mode, **env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return native.Engine(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def gpu_batched(built):
    """The batched placement path (default phase-2 variant, "slot").  Every
    variant also runs the full case list in tests/test_gpu_batch_variants.py."""
    return _engine_with_batch_mode("slot")


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


CASES = [
    ("c1-100x1000", lambda: G.config1(n_nodes=100, n_pods=1000)),   # configs[0] at full size
    ("c2-60x200", lambda: G.config2(n_nodes=60, n_pods=200)),
    ("c2-tight", lambda: G.config2(n_nodes=7, n_pods=120, seed=11)),
    ("c2-1000x1500", lambda: G.config2(n_nodes=1000, n_pods=1500)),
    ("c2-most-allocated", lambda: (lambda n, p, _: (n, p, P.config2_profile(strategy=P.MOST_ALLOCATED)))(
        *G.config2(n_nodes=300, n_pods=600, seed=12))),
    ("c5-small", lambda: G.config5(n_nodes=400, n_pods=300, n_images=200, taint_vocab=128,
                                   taints_per_node=16, images_per_node=20)),
    ("readme-kat", G.readme_kat),
    ("readme-kat2", G.readme_kat2),
    ("c3-60x400", lambda: G.config3(n_nodes=60, n_pods=400, apps=12, zones=4)),
    ("c3-600x3000", lambda: G.config3(n_nodes=600, n_pods=3000, apps=40, zones=8)),
] + [(f"zoo-{s}", (lambda s=s: __import__("zoo").zoo(s))) for s in range(8)] + [
    # plugin args beyond the defaults (parity unpinned against Go: both oracles only)
    ("c2-rtcr-1000x1500", lambda: _with_rtcr(*G.config2(n_nodes=1000, n_pods=1500, seed=13),
                                             [(0, 2), (30, 9), (70, 10), (100, 1)])),
] + [(f"zoo-{k}-{s}", (lambda s=s, k=k: __import__("zoo").zoo_args(s, k)))
     for k in ("rtcr", "pts-list") for s in range(3)]


def _with_rtcr(nodes, pods, prof, shape):
    prof.fit_strategy = P.REQUESTED_TO_CAPACITY_RATIO
    prof.fit_shape = shape
    return nodes, pods, prof


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_queue_capture_matches_oracle(gpu, oracle, name, make):
    nodes, pods, prof = make()
    enc = E.Encoder(nodes, pods, prof)
    pl = compare_engine_runs(enc, prof, gpu, oracle, name)
    # node state after the queue
    R = len(enc.cluster.res_names)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    assert (pl >= 0).any()


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_placement_queue_matches_oracle(gpu_batched, oracle, name, make):
    """Placement-only queue (no capture): the batched speculate-and-repair path."""
    gpu = gpu_batched
    nodes, pods, prof = make()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    pg, rg = gpu.run_queue(0, len(pods))
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pg, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    R = len(enc.cluster.res_names)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    # second half of the queue after a reset + split: batches straddling calls
    gpu.reset_state()
    half = len(pods) // 2
    p1, _ = gpu.run_queue(0, half)
    p2, _ = gpu.run_queue(half, len(pods) - half)
    np.testing.assert_array_equal(np.concatenate([p1, p2]), po)


def test_readme_kat2_gpu(gpu, gpu_batched):
    """The second reference-held vector (plugin-extender.md:85-107, tests/
    test_kat.py): the per-cycle path (ksg_eval + ksg_commit, as the cgo shim
    drives it) and the batched captured queue both give node-282x7 Fit 47 /
    BalancedAllocation 52, node-gp9t4 73 / 76, and select node-gp9t4."""
    from test_kat import KAT2, KAT2_SELECTED
    nodes, pods, prof = G.readme_kat2()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    names = enc.cluster.node_names
    gpu.load(enc, pf)
    r0 = gpu.eval(0)
    assert names[r0.selected] == "node-282x7"
    gpu.commit(0, r0.selected)
    cap = native.CaptureBuffers(2, 1)
    r1 = gpu.eval(1, cap)
    assert r1.n_feasible == 2 and names[r1.selected] == KAT2_SELECTED
    for n, node in enumerate(names):
        assert cap.raw[0, P.NODE_RESOURCES_FIT, n] == KAT2[node]["NodeResourcesFit"]
        assert cap.raw[0, P.BALANCED_ALLOCATION, n] == KAT2[node]["NodeResourcesBalancedAllocation"]
    for eng in (gpu, gpu_batched):
        eng.load(enc, pf)
        capq = native.CaptureBuffers(2, 2)
        pl, _ = eng.run_queue(0, 2, capture=capq)
        assert [names[x] for x in pl] == ["node-282x7", KAT2_SELECTED]
        for n, node in enumerate(names):
            assert capq.raw[1, P.NODE_RESOURCES_FIT, n] == KAT2[node]["NodeResourcesFit"]
            assert capq.raw[1, P.BALANCED_ALLOCATION, n] == KAT2[node]["NodeResourcesBalancedAllocation"]


@pytest.mark.parametrize("seed", [0, 3, 5])
def test_zoo_annotation_bytes_gpu_vs_pyoracle(gpu, seed):
    from zoo import zoo
    nodes, pods, prof = zoo(seed, n_pods=80)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, gpu)
    assert want == got


@pytest.mark.parametrize("kind,seed", [("rtcr", 0), ("rtcr", 2), ("pts-list", 0), ("pts-list", 1)])
def test_zoo_plugin_args_annotation_bytes_gpu_vs_pyoracle(gpu, kind, seed):
    """RequestedToCapacityRatio / PodTopologySpread defaultConstraints: every
    annotation byte from the GPU equals the Python restatement's (parity
    unpinned against Go: no reference fixture covers these args)."""
    from zoo import zoo_args
    nodes, pods, prof = zoo_args(seed, kind, n_pods=80)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, gpu)
    assert want == got


def test_annotations_bytes_gpu_vs_pyoracle(gpu):
    nodes, pods, prof = G.config2(n_nodes=40, n_pods=60, seed=21)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, gpu)
    assert want == got


def test_eval_does_not_commit_and_commit_matches(gpu, oracle):
    nodes, pods, prof = G.config2(n_nodes=200, n_pods=50, seed=5)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    R = len(enc.cluster.res_names)
    before = gpu.read_state(R)
    r1 = gpu.eval(3)
    r2 = gpu.eval(3)
    assert r1.selected == r2.selected and r1.n_feasible == r2.n_feasible
    for a, b in zip(before, gpu.read_state(R)):
        np.testing.assert_array_equal(a, b)
    for i in range(20):   # host-driven cycle: eval + commit, as the cgo shim does
        g, o = gpu.eval(i), oracle.eval(i)
        assert (g.selected, g.n_feasible, g.status) == (o.selected, o.n_feasible, o.status)
        if g.selected >= 0:
            gpu.commit(i, g.selected)
            oracle.commit(i, o.selected)
    for a, b in zip(gpu.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)
    gpu.reset_state()
    for a, b in zip(before, gpu.read_state(R)):
        np.testing.assert_array_equal(a, b)


def test_replicas_match_sequential_oracle(gpu, oracle):
    nodes, pods, base = G.config2(n_nodes=150, n_pods=300, seed=2)
    enc = E.Encoder(nodes, pods, base)
    profs = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(6)]
    gpu.load(enc, profs[0])
    oracle.load(enc, profs[0])
    pl, sums = gpu.run_replicas(profs, 0, len(pods))
    want, wsums = oracle.run_replicas(profs, 0, len(pods))
    np.testing.assert_array_equal(pl, want)
    assert (sums["scheduled"] + sums["unschedulable"] == len(pods)).all()
    for f in wsums.dtype.names:
        np.testing.assert_array_equal(sums[f], wsums[f], err_msg=f)
    # the sweep entry point (world 1: no collective) returns the same
    replicas = pkg("replicas")
    spl, ssm = replicas.run_sweep(gpu, profs, 0, len(pods))
    np.testing.assert_array_equal(spl, want)
    np.testing.assert_array_equal(ssm[:, 0], wsums["scheduled"])
    # replicas start from (and do not modify) the context's own state
    R = len(enc.cluster.res_names)
    assert int(gpu.read_state(R)[2].sum()) == 0


@pytest.mark.slow
def test_full_config2_placements(gpu_batched, oracle):
    """BASELINE configs[1] at full size: 5,000 nodes x 50,000 pods."""
    gpu = gpu_batched
    nodes, pods, prof = G.config2()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    pg, rg = gpu.run_queue(0, len(pods))
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pg, po)
    np.testing.assert_array_equal(rg["n_feasible"], ro["n_feasible"])


def test_kernel_timing_accounts_for_the_run(gpu_batched):
    """ksg_set_timing: per-kernel HIP-event durations cover the run (bench.py's roofline input)."""
    gpu = gpu_batched
    nodes, pods, prof = G.config2(n_nodes=500, n_pods=700, seed=9)
    enc = E.Encoder(nodes, pods, prof)
    gpu.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    gpu.set_timing(True)
    gpu.run_queue(0, len(pods), results=False)
    stats = {k["name"]: k for k in gpu.kernel_stats()}
    gpu.set_timing(False)
    assert {"ksg_batch_phase1", "ksg_batch_topk", "ksg_batch_phase2s"} <= set(stats)
    assert stats["ksg_batch_phase1"]["units"] == len(pods) * len(nodes)
    total = sum(k["total_ms"] for k in stats.values())
    assert 0 < total <= gpu.last_kernel_ms() * 1.05 + 0.05
