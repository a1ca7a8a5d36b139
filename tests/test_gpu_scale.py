"""BASELINE configs[3] and configs[4] at their defining launch shapes
(ksg_run_replicas), bit-exact against the C++ oracle.

* configs[3]: 1,024 what-if replicas x 5,000 nodes (the config-2 cluster and
  queue), per-replica weights and strategies from G.replica_profiles: all
  1,024 replicas resident at once, four 256-lane workgroups per CU.  The
  placements of 16 evenly spaced replicas and the summaries (scheduled /
  unschedulable counts, placement hash, Σ requested cpu / memory) of ALL
  1,024 replicas are compared with the oracle.
* configs[4]: 100,000 nodes, 64 taints per node from a 1,024-entry
  vocabulary, 10,000 images, amd.com/gpu on 30 % of nodes, 64 replicas: the
  host picks S = 8 workgroups per replica with the per-node results in the
  per-replica scratch row (12,500 nodes per workgroup exceed the register
  budget).  Every replica's placements and summary are compared.

The queue is a prefix of the full one (the oracle has to finish in seconds);
the launch shape does not depend on the queue length."""
import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
P = pkg("profile")
native = pkg("native")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(built):
    return native.Engine(device=0)


@pytest.fixture(scope="module")
def oracle():
    import binding
    return binding.Oracle(16)


def _compare(pl, sums, want, wsums, rows):
    for k, r in enumerate(rows):
        bad = np.nonzero(pl[r] != want[k])[0]
        assert bad.size == 0, f"replica {r}: first mismatches at pods {bad[:5]}: gpu {pl[r][bad[:5]]} " \
                              f"oracle {want[k][bad[:5]]}"


def test_config4_1024_replicas(gpu, oracle):
    R, PODS = 1024, 200
    nodes, pods, base, rprofs = G.config4(n_replicas=R, n_pods=PODS)
    enc = E.Encoder(nodes, pods, base)
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in rprofs]
    gpu.load(enc, pf[0])
    pl, sums = gpu.run_replicas(pf, 0, PODS)
    oracle.load(enc, pf[0])
    # every replica's summary ...
    _, wsums = oracle.run_replicas(pf, 0, PODS)
    for f in wsums.dtype.names:
        bad = np.nonzero(sums[f] != wsums[f])[0]
        assert bad.size == 0, f"summary field {f}: replicas {bad[:8]} differ"
    # ... and the full placements of 16 evenly spaced replicas
    rows = sorted(set(np.linspace(0, R - 1, 16).astype(int).tolist()))
    want, _ = oracle.run_replicas([pf[r] for r in rows], 0, PODS)
    _compare(pl, sums, want, None, rows)
    assert (sums["scheduled"] == PODS).all()
    # the what-if profiles really lead to different placements
    assert len(set(sums["placement_hash"].tolist())) > 16


def test_config5_100k_nodes_s8(gpu, oracle):
    R, PODS = 64, 100
    nodes, pods, base = G.config5(n_pods=PODS)
    enc = E.Encoder(nodes, pods, base)
    assert enc.cluster.max_taints == 64 and enc.cluster.n_images > 9000
    plist = []
    for r in range(R):
        plugins = [(n, (w + r % 3) if w else 0) for n, w in base.plugins]
        plist.append(P.Profile(plugins=plugins, fit_strategy=r % 2, fit_resources=base.fit_resources,
                               ba_resources=base.ba_resources))
    pf = [E.encode_profile(p, enc.cluster.res_names) for p in plist]
    gpu.load(enc, pf[0])
    pl, sums = gpu.run_replicas(pf, 0, PODS)
    oracle.load(enc, pf[0])
    want, wsums = oracle.run_replicas(pf, 0, PODS)
    _compare(pl, sums, want, wsums, list(range(R)))
    for f in wsums.dtype.names:
        np.testing.assert_array_equal(sums[f], wsums[f], err_msg=f)
    assert (pl >= 0).mean() > 0.9
