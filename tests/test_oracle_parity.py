"""CPU-side parity: the pure-Python restatement (object model) against the C++
oracle (encoded form), including every byte of the annotations the wrapped
plugins record."""
import pytest

from conftest import pkg
from helpers import pyoracle_annotations, scheduler_annotations

G = pkg("generator")


CASES = [
    ("c1", lambda: G.config1(n_nodes=30, n_pods=80)),
    ("c2", lambda: G.config2(n_nodes=50, n_pods=120)),
    ("c2-tight", lambda: G.config2(n_nodes=6, n_pods=90, seed=7)),
]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_annotations_pyoracle_vs_oracle(name, make):
    import binding
    nodes, pods, prof = make()
    want, recs = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(2))
    for i, (w, g) in enumerate(zip(want, got)):
        assert w == g, f"{name}: pod {i} annotations differ"
    assert any(r["n_feasible"] == 0 for r in recs) or name != "c2-tight"


def test_readme_kat_annotation_bytes():
    import binding
    nodes, pods, prof = G.readme_kat()
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(1))[0]
    A = pkg("annotations")
    assert got[A.SCORE] == ('{"node-282x7":{"ImageLocality":"0","NodeResourcesBalancedAllocation":"76",'
                            '"NodeResourcesFit":"73","TaintToleration":"0"},"node-gp9t4":{"ImageLocality":"0",'
                            '"NodeResourcesBalancedAllocation":"76","NodeResourcesFit":"73","TaintToleration":"0"}}')
    assert '"TaintToleration":"300"' in got[A.FINALSCORE]
    assert got[A.SELECTED_NODE] == "node-282x7"
    assert got[A.BIND] == '{"DefaultBinder":"success"}'
    assert got[A.RESERVE] == '{"VolumeBinding":"success"}'


@pytest.mark.parametrize("seed", range(6))
def test_zoo_annotations_pyoracle_vs_oracle(seed):
    """Randomised edge-case workloads (tests/zoo.py): every byte of every
    annotation from the C++ oracle equals the pure-Python restatement."""
    import binding
    from zoo import zoo
    nodes, pods, prof = zoo(seed)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(2))
    for i, (w, g) in enumerate(zip(want, got)):
        assert w == g, f"zoo seed {seed}: pod {i} annotations differ"


@pytest.mark.parametrize("kind", ["rtcr", "pts-list"])
@pytest.mark.parametrize("seed", range(3))
def test_zoo_plugin_args_pyoracle_vs_oracle(kind, seed):
    """RequestedToCapacityRatio and PodTopologySpread defaultConstraints
    (tests/zoo.py zoo_args): both restatements agree byte for byte.  Parity
    unpinned against Go: no reference fixture covers these args."""
    import binding
    from zoo import zoo_args
    nodes, pods, prof = zoo_args(seed, kind)
    want, recs = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(2))
    for i, (w, g) in enumerate(zip(want, got)):
        assert w == g, f"zoo {kind} seed {seed}: pod {i} annotations differ"
    assert any(r["n_feasible"] >= 2 for r in recs)


def test_config3_small_annotations():
    import binding
    nodes, pods, prof = G.config3(n_nodes=40, n_pods=200, apps=10, zones=4)
    want, _ = pyoracle_annotations(nodes, pods, prof)
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(2))
    assert want == got
