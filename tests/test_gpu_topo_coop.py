"""GPU parity of the chip-wide PodTopologySpread / InterPodAffinity path
(ksg_topo_coop): G workgroups share each pod through grid
barriers.  Placements, per-pod results and the node state after the queue are
compared bit for bit with the C++ oracle at sizes that spread a pod over many
workgroups (G = N / 256), including the zoo's edge cases (several soft
constraints: the extra-barrier branch; minDomains; namespaces; existing pods'
terms) and split calls."""
import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[(0, 1), (1, 1), (0, 0)], ids=["atomic-merge", "partial-slots", "pod-by-pod"])
def gpu(built, request):
    """Both histogram hand-offs (KSG_COOP_PMODE, read at ksg_open): 0 (default)
    merges each workgroup's partial histograms into an accumulator with
    agent-scope atomics, 1 folds every workgroup's partial slot; placement
    runs take the speculative topology queue (windows of independent pods,
    ksched_topo_win.h, the default since round 6), or ksg_topo_coop pod by
    pod (KSG_TOPO_WINDOW=0)."""
    import os
    pmode, window = request.param
    env = {"KSG_COOP_PMODE": str(pmode), "KSG_TOPO_WINDOW": str(window)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = native.Engine(device=0)
        eng.window = bool(window)
        return eng
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


CASES = [
    ("c3-4000x1200", lambda: G.config3(n_nodes=4000, n_pods=1200, apps=60, zones=8)),
    ("c3-15000x300", lambda: G.config3(n_nodes=15000, n_pods=300)),
    # configs[2]'s full cluster with a queue long enough for domains to fill
    # (every zone holds pods of the big apps, hostname spreads bind)
    ("c3-15000x3000", lambda: G.config3(n_nodes=15000, n_pods=3000)),
    ("c1-2000x800", lambda: G.config1(n_nodes=2000, n_pods=800)),
] + [(f"zoo-big-{s}", (lambda s=s: __import__("zoo").zoo(s, n_nodes=700, n_pods=400, apps=7, zones=5)))
     for s in range(4)] + [
    # defaultingType List: hard and soft default constraints on the owned pods
    (f"zoo-big-pts-list-{s}", (lambda s=s: __import__("zoo").zoo_args(s, "pts-list", n_nodes=700, n_pods=400,
                                                                      apps=7, zones=5))) for s in range(2)]


_ORACLE = {}   # case -> (workload, oracle placements, results, final state): both hand-offs compare to one run


def _case(oracle, name, make):
    if name not in _ORACLE:
        nodes, pods, prof = make()
        enc = E.Encoder(nodes, pods, prof)
        pf = E.encode_profile(prof, enc.cluster.res_names)
        oracle.load(enc, pf)
        po, ro = oracle.run_queue(0, len(pods))
        R = len(enc.cluster.res_names)
        ro = {f: np.array(ro[f]) for f in ("n_feasible", "status", "score_skip")}
        _ORACLE[name] = (enc, pf, len(pods), np.array(po), ro, [np.array(x) for x in oracle.read_state(R)])
    return _ORACLE[name]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_topo_coop_matches_oracle(gpu, oracle, name, make):
    enc, pf, P, po, ro, ostate = _case(oracle, name, make)
    gpu.load(enc, pf)
    pg, rg = gpu.run_queue(0, P)
    path, flags = gpu.last_run_info()
    if path == 4:   # (configs[0]'s pods need no topology kernel: the batched path)
        assert bool(flags & native.RUN_TOPO_WINDOW) == gpu.window, (path, flags)
    bad = np.nonzero(pg != po)[0]
    assert bad.size == 0, f"{name}: first mismatches at pods {bad[:5]}: gpu {pg[bad[:5]]} oracle {po[bad[:5]]}"
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    R = len(enc.cluster.res_names)
    for a, b in zip(gpu.read_state(R), ostate):
        np.testing.assert_array_equal(a, b)
    gpu.reset_state()
    third = P // 3
    p1, _ = gpu.run_queue(0, third)
    p2, _ = gpu.run_queue(third, P - third)
    np.testing.assert_array_equal(np.concatenate([p1, p2]), po)


@pytest.mark.parametrize("n_pods,tables", [(30000, "1"), (30000, "0"), (150000, "1")],
                         ids=["30k-tables", "30k-pre-pass", "150k-tables"])
def test_configs2_golden(built, n_pods, tables):
    """configs[2]'s full 15,000-node cluster against the C++ oracle's
    placements, per-pod results and final pod counts
    (tests/golden/c3_15000x<P>.npz, tests/golden/make_c3_large.py: the oracle
    takes minutes to hours at these sizes): a 30,000-pod queue with the
    maintained domain tables and their one-pod lag, and with the pre-pass path
    (KSG_COOP_TABLES=0); and BASELINE.json's full 150,000-pod queue."""
    import os
    gold = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"c3_15000x{n_pods}.npz"))
    nodes, pods, prof = G.config3(n_nodes=15000, n_pods=n_pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    old = os.environ.get("KSG_COOP_TABLES")
    os.environ["KSG_COOP_TABLES"] = tables
    try:
        eng = native.Engine(device=0)
    finally:
        if old is None:
            del os.environ["KSG_COOP_TABLES"]
        else:
            os.environ["KSG_COOP_TABLES"] = old
    eng.load(enc, pf)
    pg, rg = eng.run_queue(0, len(pods))
    # the speculative topology queue needs the maintained tables
    assert bool(eng.last_run_info()[1] & native.RUN_TOPO_WINDOW) == (tables == "1")
    bad = np.nonzero(pg != gold["placements"])[0]
    assert bad.size == 0, f"first mismatches at pods {bad[:5]}: gpu {pg[bad[:5]]} oracle {gold['placements'][bad[:5]]}"
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(np.asarray(rg[f]).astype(gold[f].dtype), gold[f], err_msg=f)
    np.testing.assert_array_equal(eng.read_state(len(enc.cluster.res_names))[2], gold["pod_count"])


@pytest.mark.parametrize("k", [2, 5])
def test_topo_window_sizes(built, oracle, k):
    """Windows of at most k pods (KSG_TOPO_WINDOW_K) place exactly as the
    oracle; the walk ends some windows early (a changed node left a pod's
    feasible set) on a cluster tight enough to fill nodes."""
    import os
    enc, pf, P, po, ro, ostate = _case(oracle, "c3-4000x1200", CASES[0][1])
    os.environ["KSG_TOPO_WINDOW_K"] = str(k)
    try:
        eng = native.Engine(device=0)
    finally:
        del os.environ["KSG_TOPO_WINDOW_K"]
    eng.load(enc, pf)
    pg, rg = eng.run_queue(0, P)
    assert eng.last_run_info()[1] & native.RUN_TOPO_WINDOW
    windows, decided, cut = eng.topo_window_stats()
    assert decided == P and P / k <= windows <= P, (windows, decided, cut)
    np.testing.assert_array_equal(pg, po)
    for f in ("n_feasible", "status", "score_skip"):
        np.testing.assert_array_equal(rg[f], ro[f], err_msg=f)
    for a, b in zip(eng.read_state(len(enc.cluster.res_names)), ostate):
        np.testing.assert_array_equal(a, b)
