"""Bulk annotation (bulk.annotate_queue): one captured run + ksg_annotate per
pod gives the same filter-result / score-result / finalscore-result bytes as
the per-pod DebuggableScheduler cycle.  CPU: the C++ oracle as the engine;
GPU (marked): libksched.so on the batched capture path."""
import threading

import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
F = pkg("framework")
A = pkg("annotations")
B = pkg("bulk")
native = pkg("native")


def _per_pod(nodes, pods, prof, engine):
    s = F.DebuggableScheduler(nodes, pods, prof, engine=engine)
    out = []
    for i in range(len(pods)):
        s.schedule_one(i)
        a = s.annotations(i)
        out.append((a[A.FILTER], a[A.SCORE], a[A.FINALSCORE]))
    return out


def _bulk(nodes, pods, prof, engine, threads, chunk):
    enc = E.Encoder(nodes, pods, prof)
    engine.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    bulk = B.BulkAnnotator(enc, prof, threads=threads)
    got = [None] * len(pods)
    lock = threading.Lock()

    def sink(i, vals):
        with lock:
            got[i] = tuple(bytes(v).decode("utf-8") for v in vals)

    try:
        pl = B.annotate_queue(engine, bulk, 0, len(pods), sink, chunk=chunk)
    finally:
        bulk.close()
    return pl, got


CASES = {
    "c2": lambda: G.config2(n_nodes=40, n_pods=90, seed=21),
    "c1-default": lambda: G.config1(n_nodes=30, n_pods=80),
    "kat": G.readme_kat,
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_bulk_matches_per_pod_oracle(name):
    import binding
    nodes, pods, prof = CASES[name]()
    want = _per_pod(nodes, pods, prof, binding.Oracle(2))
    _, got = _bulk(nodes, pods, prof, binding.Oracle(2), threads=3, chunk=32)
    assert got == want


GPU_CASES = {
    "c2-300x400": lambda: G.config2(n_nodes=300, n_pods=400, seed=21),
    "c1-default-200x300": lambda: G.config1(n_nodes=200, n_pods=300),
    "c5-small": lambda: G.config5(n_nodes=200, n_pods=150, n_images=100, taint_vocab=64, taints_per_node=8,
                                  images_per_node=10),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GPU_CASES))
def test_bulk_matches_per_pod_gpu(built, name):
    nodes, pods, prof = GPU_CASES[name]()
    want = _per_pod(nodes, pods, prof, native.Engine(device=0))
    eng = native.Engine(device=0)
    eng.set_timing(True)
    _, got = _bulk(nodes, pods, prof, eng, threads=4, chunk=128)
    assert "ksg_capture_eval" in {k["name"] for k in eng.kernel_stats()}
    assert got == want
