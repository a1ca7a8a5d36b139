"""Grid-barrier kernels: their cooperative launches and the recovery from a
barrier timeout.

The chip-wide topology kernel (queue runs and the one-pod per-cycle
evaluation), the multi-workgroup replica sweep (S > 1) and the per-cycle
kernels (one launch per cycle, the persistent server) launch plainly with a
grid inside the occupancy API's co-resident count and bound their barrier
polls.  A timeout means a workgroup was not resident: the library restores the
node state the call started from (the partial commits of a topology queue),
switches the context to cooperative launches and runs the same call again
(ksg_recoveries counts it).

* the cooperative forms (KSG_COOP_LAUNCH=1, KSG_CYCLE_COOP=1) against the
  C++ oracle, as the plain forms are in test_gpu_topo_coop / test_gpu_sweep /
  test_gpu_eval;
* a forced timeout (KSG_TEST_INJECT_TIMEOUT: the launch's sticky timeout word
  set before it starts, so its barriers give up for real; for a queue run
  the second launch, after 64 committed pods) still gives the oracle's result,
  with one recovery counted."""
import numpy as np
import pytest

from conftest import pkg
from test_gpu_eval import _check_cycles

G = pkg("generator")
E = pkg("encoder")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


def _engine(monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    return native.Engine(device=0)


def _topo_queue(eng, oracle, n_nodes=4000, n_pods=600):
    nodes, pods, prof = G.config3(n_nodes=n_nodes, n_pods=n_pods, apps=60, zones=8)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng.load(enc, pf)
    oracle.load(enc, pf)
    # a first call on the plain (or cooperative) path, then the rest
    first = 100
    pg = np.concatenate([eng.run_queue(0, first)[0], eng.run_queue(first, n_pods - first)[0]])
    po = np.concatenate([oracle.run_queue(0, first)[0], oracle.run_queue(first, n_pods - first)[0]])
    bad = np.nonzero(pg != po)[0]
    assert bad.size == 0, f"first mismatches at pods {bad[:5]}: gpu {pg[bad[:5]]} oracle {po[bad[:5]]}"
    assert eng.last_run_info()[0] == 4   # the chip-wide topology path
    R = len(enc.cluster.res_names)
    for a, b in zip(eng.read_state(R), oracle.read_state(R)):
        np.testing.assert_array_equal(a, b)


def _sweep(eng, oracle):
    nodes, pods, base = G.config2(n_nodes=5000, n_pods=150, seed=2)   # S = 2 workgroups per replica
    enc = E.Encoder(nodes, pods, base)
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(8)]
    eng.load(enc, pf[0])
    oracle.load(enc, pf[0])
    pl, sums = eng.run_replicas(pf, 0, len(pods))
    want, wsums = oracle.run_replicas(pf, 0, len(pods))
    np.testing.assert_array_equal(pl, want)
    for f in wsums.dtype.names:
        np.testing.assert_array_equal(sums[f], wsums[f], err_msg=f)
    assert eng.last_run_info()[0] == 3


def _cycles(eng, oracle, name):
    from test_gpu_eval import CASES
    _check_cycles(eng, oracle, name, *CASES[name]())


# ---- the cooperative launches ------------------------------------------------------

def test_coop_topology_queue(oracle, monkeypatch):
    eng = _engine(monkeypatch, KSG_COOP_LAUNCH=1)
    try:
        _topo_queue(eng, oracle)
        assert eng.recoveries() == 0
    finally:
        eng.close()


def test_coop_topology_one_pod(oracle, monkeypatch):
    eng = _engine(monkeypatch, KSG_COOP_LAUNCH=1)
    try:
        _cycles(eng, oracle, "c3-15000x40")
        assert eng.recoveries() == 0
    finally:
        eng.close()


def test_coop_replica_sweep(oracle, monkeypatch):
    eng = _engine(monkeypatch, KSG_COOP_LAUNCH=1)
    try:
        _sweep(eng, oracle)
    finally:
        eng.close()


@pytest.mark.parametrize("server", [0, 1], ids=["launch", "server"])
def test_coop_cycle(oracle, monkeypatch, server):
    eng = _engine(monkeypatch, KSG_CYCLE_COOP=1, KSG_CYCLE_SERVER=server)
    try:
        _cycles(eng, oracle, "c2-1000x120")
        _cycles(eng, oracle, "c1-100x150")
        assert eng.recoveries() == 0
    finally:
        eng.close()


# ---- a forced timeout: restore, cooperative relaunch, the oracle's result ------------

@pytest.mark.parametrize("window", [1, 0], ids=["windows", "pod-by-pod"])
def test_timeout_topology_queue_recovers(oracle, monkeypatch, window):
    """A barrier of the first call times out after pods were committed (pod by
    pod: the second launch, after 64 pods; the speculative topology queue:
    the rows of the 17th window): the call restores the pre-call state and
    runs again cooperatively (pod by pod from then on)."""
    eng = _engine(monkeypatch, KSG_TEST_INJECT_TIMEOUT=1, KSG_TOPO_WINDOW=window)
    try:
        _topo_queue(eng, oracle)
        assert eng.recoveries() == 1
        assert not eng.last_run_info()[1] & native.RUN_TOPO_WINDOW   # cooperative launches: pod by pod
    finally:
        eng.close()


def test_timeout_topology_one_pod_recovers(oracle, monkeypatch):
    eng = _engine(monkeypatch, KSG_TEST_INJECT_TIMEOUT=2)
    try:
        _cycles(eng, oracle, "c3-15000x40")
        assert eng.recoveries() == 1
    finally:
        eng.close()


def test_persistent_walk_recovers(oracle, monkeypatch):
    """The persistent spec walk gives up waiting for a top-k (injected: its
    give-up word set after batch 0): the call restores the pre-call state and
    runs the per-batch form (from then on), equal to the oracle."""
    eng = _engine(monkeypatch, KSG_TEST_INJECT_TIMEOUT=16)
    try:
        nodes, pods, prof = G.config2(n_nodes=1500, n_pods=1000, seed=21)
        enc = E.Encoder(nodes, pods, prof)
        pf = E.encode_profile(prof, enc.cluster.res_names)
        eng.load(enc, pf)
        oracle.load(enc, pf)
        pg, rg = eng.run_queue(0, len(pods))
        po, ro = oracle.run_queue(0, len(pods))
        np.testing.assert_array_equal(pg, po)
        for f in ("n_feasible", "status", "score_skip"):
            np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
        R = len(enc.cluster.res_names)
        for x, y in zip(eng.read_state(R), oracle.read_state(R)):
            np.testing.assert_array_equal(x, y)
        assert eng.recoveries() == 1
        assert eng.last_run_info()[1] & native.RUN_SPEC
    finally:
        eng.close()


def test_timeout_replica_sweep_recovers(oracle, monkeypatch):
    eng = _engine(monkeypatch, KSG_TEST_INJECT_TIMEOUT=4)
    try:
        _sweep(eng, oracle)
        assert eng.recoveries() == 1
    finally:
        eng.close()


def test_timeout_cycle_recovers(oracle, monkeypatch):
    """The per-cycle kernel's exchange gives up on the first cycle (its
    deferred assume and staged append already applied): the cycle is
    evaluated again cooperatively, the rest run cooperatively."""
    eng = _engine(monkeypatch, KSG_TEST_INJECT_TIMEOUT=8, KSG_CYCLE_SERVER=0)   # (the one-launch form)
    try:
        _cycles(eng, oracle, "c2-1000x120")
        assert eng.recoveries() == 1
    finally:
        eng.close()
