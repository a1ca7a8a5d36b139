"""The reference's export sample through the GPU:
simulator/docs/api-samples/v1/export.md's scheduler configuration (per-point
plugin sets, PodTopologySpread weight 2 at the Score point; the three legacy
volume-limit plugins the simulator's registry lacks removed, see
test_ingest.py) with its priority classes, plus a synthetic cluster written as
a ResourcesForSnap document, loaded by ingest.load_snapshot and scheduled on
the device.  Checks: annotation bytes of every pod against pyoracle (the
store uses the MultiPoint weights, the selection the Score point's), and
placements / result words against the C++ oracle."""
import numpy as np
import pytest

from conftest import pkg
from helpers import pyoracle_annotations, scheduler_annotations
from test_ingest import _export, export_config_loadable

G = pkg("generator")
E = pkg("encoder")
I = pkg("ingest")
P = pkg("profile")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(built):
    return native.Engine(device=0)


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


def _snapshot(make):
    nodes, pods, _ = make()
    doc = I.snapshot_document(nodes, pods, P.default_profile())
    src = _export("case2")
    doc["schedulerConfig"] = export_config_loadable()
    doc["priorityClasses"] = src["priorityClasses"]
    return I.load_snapshot(doc)


CASES = {
    "c3-40x150": lambda: G.config3(n_nodes=40, n_pods=150, apps=8, zones=4),
    "c1-60x200": lambda: G.config1(n_nodes=60, n_pods=200),
    "c2-50x120": lambda: G.config2(n_nodes=50, n_pods=120, seed=21),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_export_profile_annotations_gpu_vs_pyoracle(gpu, name):
    snap = _snapshot(CASES[name])
    assert not snap.bound
    pods = [snap.pods[i] for i in snap.queue]
    want, _ = pyoracle_annotations(snap.nodes, pods, snap.profile)
    got = scheduler_annotations(snap.nodes, pods, snap.profile, gpu)
    assert want == got


@pytest.mark.parametrize("name", sorted(CASES))
def test_export_profile_queue_gpu_vs_oracle(gpu, oracle, name):
    snap = _snapshot(CASES[name])
    pods = [snap.pods[i] for i in snap.queue]
    enc = E.Encoder(snap.nodes, pods, snap.profile)
    pf = E.encode_profile(snap.profile, enc.cluster.res_names)
    gpu.load(enc, pf)
    oracle.load(enc, pf)
    pg, rg = gpu.run_queue(0, len(pods))
    po, ro = oracle.run_queue(0, len(pods))
    np.testing.assert_array_equal(pg, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    assert (pg >= 0).sum() > 0
