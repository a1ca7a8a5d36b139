"""GPU parity of the replica sweep (ksg_run_replicas): the
static-record + per-replica sweep kernels against the C++ oracle run replica by
replica, bit-exact placements and summaries.  Cases cover every (BLOCK, KN)
shape the host picks (registers: N <= 2,048 ... 32,768; scratch row: N >
32,768; S > 1 workgroups per replica from 4,096 nodes with few replicas),
the generic (non cpu/memory) profile path, mixed strategies and
weights, nodeName / unschedulable / taint / affinity edge cases from the zoo
under node-local profiles, and profiles that fall back to the queue kernel."""
import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
m = pkg("model")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(built):
    return native.Engine(device=0)


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(8)


NODE_LOCAL = [("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0), ("TaintToleration", 3),
              ("NodeAffinity", 2), ("NodeResourcesFit", 1), ("NodeResourcesBalancedAllocation", 1),
              ("ImageLocality", 1), ("DefaultBinder", 0)]


def _zoo_profiles(k):
    rng = np.random.Generator(np.random.PCG64(100 + k))
    out = []
    for r in range(k):
        plugins = [(n, int(rng.integers(1, 6)) if w else 0) for n, w in NODE_LOCAL]
        strat = P.LEAST_ALLOCATED if r % 2 == 0 else P.MOST_ALLOCATED
        out.append(P.Profile(plugins=plugins, fit_strategy=strat))
    return out


def _c2(n_nodes, n_pods, seed=2):
    nodes, pods, base = G.config2(n_nodes=n_nodes, n_pods=n_pods, seed=seed)
    return nodes, pods, base


CASES = [
    # (name, workload, replica profiles)
    ("c2-150x300-r6", lambda: _c2(150, 300), lambda: G.replica_profiles(6)),
    ("c2-tight-r4", lambda: _c2(7, 120, seed=11), lambda: G.replica_profiles(4)),
    ("c2-3000x200-r8", lambda: _c2(3000, 200), lambda: G.replica_profiles(8)),      # KN 16
    ("c2-5000x150-r8", lambda: _c2(5000, 150), lambda: G.replica_profiles(8)),      # KN 20
    ("c2-6000x80-r3", lambda: _c2(6000, 80), lambda: G.replica_profiles(3)),        # KN 24
    ("c2-8000x60-r3", lambda: _c2(8000, 60), lambda: G.replica_profiles(3)),        # KN 32
    ("c2-12000x50-r2", lambda: _c2(12000, 50), lambda: G.replica_profiles(2)),      # 512 lanes
    ("c2-20000x40-r2", lambda: _c2(20000, 40), lambda: G.replica_profiles(2)),      # 1024 lanes
    ("c2-33000x30-r2", lambda: _c2(33000, 30), lambda: G.replica_profiles(2)),      # scratch row
    ("c5-generic-r3", lambda: G.config5(n_nodes=400, n_pods=300, n_images=200, taint_vocab=128,
                                        taints_per_node=16, images_per_node=20), None),
    ("c5-generic-6000-r3", lambda: G.config5(n_nodes=6000, n_pods=60, n_images=500, taint_vocab=256,
                                             taints_per_node=16, images_per_node=20), None),   # S = 2, generic
    ("c5-ex-6000-r2", lambda: G.config5(n_nodes=6000, n_pods=80, n_images=500, taint_vocab=256,
                                        taints_per_node=16, images_per_node=20), None),   # S = 2, cpu/mem/gpu Fit
    ("c1-default-r2", lambda: G.config1(n_nodes=100, n_pods=300), None),            # PTS/IPA: queue kernel
] + [(f"zoo-{s}-r4", (lambda s=s: __import__("zoo").zoo(s)), (lambda: _zoo_profiles(4))) for s in range(6)] + [
    # RequestedToCapacityRatio replicas beside Least/MostAllocated ones (generic arithmetic)
    ("c2-3000x200-rtcr-r4", lambda: _c2(3000, 200), lambda: _rtcr_profiles(4)),
    ("zoo-1-rtcr-r3", lambda: __import__("zoo").zoo(1), lambda: _rtcr_profiles(3, NODE_LOCAL)),
]


def _rtcr_profiles(k, plugins=None):
    shapes = __import__("zoo").RTCR_SHAPES
    out = []
    for r, p in enumerate(G.replica_profiles(k)):
        if plugins is not None:
            p = P.Profile(plugins=list(plugins), fit_strategy=p.fit_strategy)
        if r % 2 == 0:
            p.fit_strategy = P.REQUESTED_TO_CAPACITY_RATIO
            p.fit_shape = list(shapes[(r // 2) % len(shapes)])
        out.append(p)
    return out


@pytest.mark.parametrize("name,make,profs", CASES, ids=[c[0] for c in CASES])
def test_sweep_matches_oracle(gpu, oracle, name, make, profs):
    nodes, pods, base = make()
    enc = E.Encoder(nodes, pods, base)
    if profs is None:   # the workload's own profile, with varied weights / strategy
        plist = []
        for r in range(3 if name.startswith("c5") else 2):
            plugins = [(n, (w + r) if w else 0) for n, w in base.plugins]
            ba = base.ba_resources
            if name.startswith("c5") and r == 2:   # BalancedAllocation over three columns: generic arithmetic
                ba = list(base.ba_resources) + [("amd.com/gpu", 1)]
            plist.append(P.Profile(plugins=plugins, fit_strategy=r % 2, fit_resources=base.fit_resources,
                                   ba_resources=ba))
    else:
        plist = profs()
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in plist]
    gpu.load(enc, pf[0])
    oracle.load(enc, pf[0])
    pl, sums = gpu.run_replicas(pf, 0, len(pods))
    want, wsums = oracle.run_replicas(pf, 0, len(pods))
    for r in range(len(pf)):
        bad = np.nonzero(pl[r] != want[r])[0]
        assert bad.size == 0, f"{name} replica {r}: first mismatch at pod {bad[:5]}: gpu {pl[r][bad[:5]]} " \
                              f"oracle {want[r][bad[:5]]}"
    for f in wsums.dtype.names:
        np.testing.assert_array_equal(sums[f], wsums[f], err_msg=f)
    assert (pl >= 0).any()


def test_sweep_queue_subrange(gpu, oracle):
    """A sub-range of the queue (batches not aligned to the first pod)."""
    nodes, pods, base = _c2(400, 300)
    enc = E.Encoder(nodes, pods, base)
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(5)]
    gpu.load(enc, pf[0])
    oracle.load(enc, pf[0])
    pl, _ = gpu.run_replicas(pf, 100, 150)
    want, _ = oracle.run_replicas(pf, 100, 150)
    np.testing.assert_array_equal(pl, want)


# ---- narrow records: 16-byte per-(replica, node) state ----

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
def wide(built):
    """The int64-column sweep instances (KSG_FORCE_PATH=3 skips the narrow records)."""
    return _engine_env(KSG_FORCE_PATH=3)


def _sweep_kernel(eng):
    names = {k["name"] for k in eng.kernel_stats()}
    assert names & {"ksg_sweep", "ksg_sweep_narrow"}, names
    return "ksg_sweep_narrow" if "ksg_sweep_narrow" in names else "ksg_sweep"


def _run(eng, oracle, nodes, pods, base, plist):
    enc = E.Encoder(nodes, pods, base)
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in plist]
    eng.load(enc, pf[0])
    oracle.load(enc, pf[0])
    pl, sums = eng.run_replicas(pf, 0, len(pods))
    want, wsums = oracle.run_replicas(pf, 0, len(pods))
    np.testing.assert_array_equal(pl, want)
    for f in wsums.dtype.names:
        np.testing.assert_array_equal(sums[f], wsums[f], err_msg=f)
    return pl


NARROW_CASES = [
    ("c2-150x300-r6", lambda: _c2(150, 300), lambda b: G.replica_profiles(6), "ksg_sweep_narrow"),
    ("c2-5000x150-r8", lambda: _c2(5000, 150), lambda b: G.replica_profiles(8), "ksg_sweep_narrow"),
    ("c2-33000x30-r2", lambda: _c2(33000, 30), lambda b: G.replica_profiles(2), "ksg_sweep_narrow"),
    ("c5-ex-6000-r2", lambda: G.config5(n_nodes=6000, n_pods=80, n_images=500, taint_vocab=256,
                                        taints_per_node=16, images_per_node=20),
     lambda b: [b, P.Profile(plugins=[(n, w + 1 if w else 0) for n, w in b.plugins], fit_strategy=1,
                             fit_resources=b.fit_resources, ba_resources=b.ba_resources)], "ksg_sweep_narrow"),
]


@pytest.mark.parametrize("name,make,profs,kernel", NARROW_CASES, ids=[c[0] for c in NARROW_CASES])
def test_narrow_sweep_runs_and_matches_wide(timed, wide, oracle, name, make, profs, kernel):
    """The narrow instances run where the ranges allow and agree bit for bit
    with the int64 instances and the oracle."""
    nodes, pods, base = make()
    plist = profs(base)
    a = _run(timed, oracle, nodes, pods, base, plist)
    assert _sweep_kernel(timed) == kernel
    b = _run(wide, oracle, nodes, pods, base, plist)
    np.testing.assert_array_equal(a, b)


def test_narrow_fallback_on_sub_mib_memory(timed, oracle):
    """One node whose memory is not a whole number of MiB: the node-side check
    (ksg_narrow_init) sends the run to the int64 instances."""
    nodes, pods, base = _c2(300, 200)
    nodes[17].allocatable[m.MEMORY] += 1000
    _run(timed, oracle, nodes, pods, base, G.replica_profiles(4))
    assert _sweep_kernel(timed) == "ksg_sweep"


def test_narrow_fallback_on_third_column(timed, oracle):
    """A pod requesting ephemeral storage: the host-side check keeps the int64
    instances (the narrow record has no column for it)."""
    nodes, pods, base = _c2(300, 200)
    pods[5].containers[0].requests[m.EPHEMERAL] = 1 << 30
    _run(timed, oracle, nodes, pods, base, G.replica_profiles(4))
    assert _sweep_kernel(timed) == "ksg_sweep"


def test_narrow_pod_count_field_at_255(timed, wide, oracle):
    """allowed pods = 255 and tiny pods: the 8-bit pod count reaches its
    maximum, after which Fit rejects the node (Too many pods)."""
    nodes, pods, base = _c2(4, 1200, seed=7)
    for n in nodes:
        n.allocatable[m.PODS] = 255
        n.taints = []
    for p in pods:
        p.containers[0].requests = {m.CPU: 1, m.MEMORY: 1 << 20}
        p.node_affinity_required = None
    a = _run(timed, oracle, nodes, pods, base, G.replica_profiles(3))
    assert _sweep_kernel(timed) == "ksg_sweep_narrow"
    assert (a >= 0).sum(axis=1).max() == 4 * 255
    b = _run(wide, oracle, nodes, pods, base, G.replica_profiles(3))
    np.testing.assert_array_equal(a, b)


def test_narrow_fallback_on_allowed_above_255(timed, oracle):
    nodes, pods, base = _c2(4, 300, seed=7)
    nodes[2].allocatable[m.PODS] = 256
    _run(timed, oracle, nodes, pods, base, G.replica_profiles(2))
    assert _sweep_kernel(timed) == "ksg_sweep"
