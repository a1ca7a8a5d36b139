"""The device annotation serialiser (ksg_run_queue_json, csrc/ksched_json.h)
against the host one (ksg_annotate over the same captured queue run): every
byte of every pod's filter-result, score-result and finalscore-result, on the
batched capture path and the chip-wide topology path."""
import numpy as np
import pytest

from conftest import pkg

pytestmark = pytest.mark.gpu

B = pkg("bulk")
E = pkg("encoder")
G = pkg("generator")
P = pkg("profile")
native = pkg("native")

CASES = {
    "c2-1000x300": lambda: G.config2(n_nodes=1000, n_pods=300, seed=4),
    "c2-tight": lambda: G.config2(n_nodes=7, n_pods=120, seed=11),
    "c2-most": lambda: (lambda n, p, _: (n, p, P.config2_profile(strategy=P.MOST_ALLOCATED)))(
        *G.config2(n_nodes=300, n_pods=200, seed=12)),
    "c1-200x300": lambda: G.config1(n_nodes=200, n_pods=300),
    "c5-small": lambda: G.config5(n_nodes=400, n_pods=150, n_images=200, taint_vocab=128, taints_per_node=16,
                                  images_per_node=20),
    "c3-300x400": lambda: G.config3(n_nodes=300, n_pods=400, apps=12, zones=4),
    "zoo-2": lambda: __import__("zoo").zoo(2),
    "zoo-rtcr-0": lambda: __import__("zoo").zoo_args(0, "rtcr"),
}


@pytest.fixture(scope="module")
def engines(built):
    a, b = native.Engine(device=0), native.Engine(device=0)
    yield a, b
    a.close()
    b.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_device_json_matches_host(engines, name):
    ea, eb = engines
    nodes, pods, prof = CASES[name]()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    bulk = B.BulkAnnotator(enc, prof, threads=1)
    try:
        host, dev = {}, {}
        ea.load(enc, pf)
        pa = B.annotate_queue(ea, bulk, 0, len(pods), lambda i, v: host.__setitem__(i, tuple(bytes(x) for x in v)),
                              chunk=128)
        eb.load(enc, pf)
        pb = B.annotate_queue_device(eb, bulk, 0, len(pods),
                                     lambda i, v: dev.__setitem__(i, tuple(bytes(x) for x in v)), chunk=128)
    finally:
        bulk.close()
    np.testing.assert_array_equal(pa, pb)
    assert sorted(host) == sorted(dev) == list(range(len(pods)))
    for i in range(len(pods)):
        for j, what in enumerate(("filter", "score", "finalscore")):
            assert host[i][j] == dev[i][j], f"{name} pod {i} {what}: host {host[i][j][:300]!r} device {dev[i][j][:300]!r}"
