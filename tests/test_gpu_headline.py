"""The headline pinned at its own size: BASELINE.json's
metric workload, the in-tree default profile (generator.config1, seed 1) at
5,000 nodes x 50,000 pods, through the same ksg_run_queue the bench times.

The expected values are the C++ oracle's placements, per-pod results and final
pod counts over the whole queue (tests/golden/c1_5000x50000.npz, written by
`python tests/golden/make_c3_large.py 8 50000 config1 5000`).  Two phase-2
forms run it: the default speculate-and-verify walk (the bench's path) and
the slot walk inside the two-stream window (the fallback the walk hands
unsupported batches to).  The default profile follows
`simulator/scheduler/scheduler_test.go:519-541` and the weights
`simulator/scheduler/plugin/plugins_test.go:183-203`."""
import os

import numpy as np
import pytest

from conftest import pkg
from test_gpu_parity import _engine_with_batch_mode

G = pkg("generator")
E = pkg("encoder")
native = pkg("native")

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1_5000x50000.npz")


@pytest.fixture(scope="module")
def workload():
    nodes, pods, prof = G.config1(n_nodes=5000, n_pods=50000)
    enc = E.Encoder(nodes, pods, prof)
    return enc, E.encode_profile(prof, enc.cluster.res_names), np.load(GOLD)


@pytest.mark.parametrize("mode", ["spec", "window"])
def test_headline_matches_oracle(built, workload, mode):
    enc, pf, gold = workload
    eng = _engine_with_batch_mode(mode)
    try:
        eng.load(enc, pf)
        for rep in range(2):   # the bench's step: reset + the whole queue, twice
            eng.reset_state()
            pg, rg = eng.run_queue(0, len(enc.workload.pods))
            bad = np.nonzero(pg != gold["placements"])[0]
            assert bad.size == 0, (f"{mode} rep {rep}: {bad.size} mismatches, first at pods {bad[:5]}: "
                                   f"gpu {pg[bad[:5]]} oracle {gold['placements'][bad[:5]]}")
            for f in ("n_feasible", "status", "score_skip"):
                np.testing.assert_array_equal(np.asarray(rg[f]).astype(gold[f].dtype), gold[f], err_msg=f)
            np.testing.assert_array_equal(eng.read_state(len(enc.cluster.res_names))[2], gold["pod_count"])
        if mode == "spec":
            path, flags = eng.last_run_info()
            assert flags & native.RUN_SPEC, f"the headline queue left the spec walk (path {path}, flags {flags:#x})"
    finally:
        eng.close()
