"""Capture on the batched placement path (ksched_capture.h):
a captured queue runs phase 1 / top-k / phase 2 and then the two capture
kernels per batch.  Every array the wrapped plugins would record (filter
status words of all nodes, raw / normalised scores of the score plugins,
totals) must equal the C++ oracle's and the single-workgroup queue kernel's
bit for bit, on every node (zeros where nothing is recorded)."""
import numpy as np
import pytest

from conftest import pkg
from helpers import capture_queue

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
native = pkg("native")

pytestmark = pytest.mark.gpu


def _engine_env(**env):
    import os
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
def timed(built):
    eng = native.Engine(device=0)
    eng.set_timing(True)
    return eng


@pytest.fixture(scope="module")
def queue_kernel(built):
    return _engine_env(KSG_FORCE_PATH=1)


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


CASES = [
    ("c2-60x200", lambda: G.config2(n_nodes=60, n_pods=200)),
    ("c2-tight", lambda: G.config2(n_nodes=7, n_pods=120, seed=11)),
    ("c2-1000x700", lambda: G.config2(n_nodes=1000, n_pods=700)),
    ("c2-most", lambda: (lambda n, p, _: (n, p, P.config2_profile(strategy=P.MOST_ALLOCATED)))(
        *G.config2(n_nodes=300, n_pods=400, seed=12))),
    ("c1-100x300", lambda: G.config1(n_nodes=100, n_pods=300)),
    ("c5-small", lambda: G.config5(n_nodes=300, n_pods=200, n_images=200, taint_vocab=64, taints_per_node=8,
                                   images_per_node=10)),
    ("readme-kat", G.readme_kat),
]


def _run(eng, enc, pf, n, N):
    eng.load(enc, pf)
    return capture_queue(eng, n, N)


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_batched_capture_matches(timed, queue_kernel, oracle, name, make):
    nodes, pods, prof = make()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    n, N = len(pods), len(nodes)
    pg, rg, cg = _run(timed, enc, pf, n, N)
    assert "ksg_capture_eval" in {k["name"] for k in timed.kernel_stats()}, "capture did not take the batched path"
    po, ro, co = _run(oracle, enc, pf, n, N)
    pq, rq, cq = _run(queue_kernel, enc, pf, n, N)
    for other, label in ((co, "oracle"), (cq, "queue kernel")):
        np.testing.assert_array_equal(cg.fstatus, other.fstatus, err_msg=f"{label}: fstatus")
        np.testing.assert_array_equal(cg.total, other.total, err_msg=f"{label}: total")
        for pid in range(native.NPLUGINS):
            if (pf["score_mask"] >> pid) & 1:
                np.testing.assert_array_equal(cg.raw[:, pid], other.raw[:, pid], err_msg=f"{label}: raw {pid}")
                np.testing.assert_array_equal(cg.norm[:, pid], other.norm[:, pid], err_msg=f"{label}: norm {pid}")
    for p in (po, pq):
        np.testing.assert_array_equal(pg, p)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)


def test_batched_capture_split_calls(timed, oracle):
    """Two captured calls in a row (state carried between them)."""
    nodes, pods, prof = G.config2(n_nodes=500, n_pods=400, seed=3)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    N = len(nodes)
    out = []
    for eng in (timed, oracle):
        eng.load(enc, pf)
        c1 = native.CaptureBuffers(N, 150)
        c2 = native.CaptureBuffers(N, 250)
        eng.run_queue(0, 150, capture=c1)
        eng.run_queue(150, 250, capture=c2)
        out.append((c1, c2))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a.fstatus, b.fstatus)
        np.testing.assert_array_equal(a.total, b.total)
        np.testing.assert_array_equal(a.raw, b.raw)
        np.testing.assert_array_equal(a.norm, b.norm)


# ---- captured topology queues on the chip-wide kernel ----
TOPO_CASES = [
    ("c3-400x300", lambda: G.config3(n_nodes=400, n_pods=300, apps=20, zones=4)),
    ("c3-3000x200", lambda: G.config3(n_nodes=3000, n_pods=200, apps=40, zones=8)),
    ("zoo-1", lambda: __import__("zoo").zoo(1, n_pods=120)),
    ("zoo-3", lambda: __import__("zoo").zoo(3, n_pods=120)),
]


@pytest.mark.parametrize("name,make", TOPO_CASES, ids=[c[0] for c in TOPO_CASES])
def test_topology_capture_on_the_chip_wide_kernel(timed, queue_kernel, oracle, name, make):
    """PodTopologySpread / InterPodAffinity pods captured by ksg_topo_coop's
    capture instance (compact rows, every node written) equal the oracle and
    the single-workgroup queue kernel on every array, every node."""
    nodes, pods, prof = make()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    n, N = len(pods), len(nodes)
    pg, rg, cg = _run(timed, enc, pf, n, N)
    names = {k["name"] for k in timed.kernel_stats()}
    assert any("ksg_topo_coop" in k for k in names), names
    po, ro, co = _run(oracle, enc, pf, n, N)
    pq, rq, cq = _run(queue_kernel, enc, pf, n, N)
    for other, label in ((co, "oracle"), (cq, "queue kernel")):
        np.testing.assert_array_equal(cg.fstatus, other.fstatus, err_msg=f"{label}: fstatus")
        np.testing.assert_array_equal(cg.total, other.total, err_msg=f"{label}: total")
        for pid in range(native.NPLUGINS):
            if (pf["score_mask"] >> pid) & 1:
                np.testing.assert_array_equal(cg.raw[:, pid], other.raw[:, pid], err_msg=f"{label}: raw {pid}")
                np.testing.assert_array_equal(cg.norm[:, pid], other.norm[:, pid], err_msg=f"{label}: norm {pid}")
    for p in (po, pq):
        np.testing.assert_array_equal(pg, p)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
