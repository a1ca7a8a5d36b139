"""Native result-store serialiser (ksg_annotate)
against the Python Store mirror: byte-identical annotations on every workload
family, with the C++ oracle as the evaluator (CPU).  The serialiser is host
code inside libksched.so, so these tests need no GPU."""
import time

import pytest

from conftest import pkg

G = pkg("generator")
F = pkg("framework")
A = pkg("annotations")
native = pkg("native")

WORKLOADS = {
    "readme-kat": G.readme_kat,
    "c1": lambda: G.config1(n_nodes=40, n_pods=120),
    "c2": lambda: G.config2(n_nodes=60, n_pods=120, seed=21),
    "c2-tight": lambda: G.config2(n_nodes=7, n_pods=120, seed=11),
    "c3": lambda: G.config3(n_nodes=40, n_pods=150, apps=8, zones=4),
    "c5": lambda: G.config5(n_nodes=60, n_pods=40, n_images=50, taint_vocab=64, taints_per_node=8,
                            images_per_node=10),
}


def _annotations(nodes, pods, prof, native_annotations):
    import binding
    s = F.DebuggableScheduler(nodes, pods, prof, engine=binding.Oracle(2), native_annotations=native_annotations)
    out = []
    for i in range(len(pods)):
        s.schedule_one(i)
        out.append(s.annotations(i))
    return out


@pytest.mark.parametrize("name", sorted(WORKLOADS))
def test_native_serialiser_matches_store(built, name):
    nodes, pods, prof = WORKLOADS[name]()
    assert _annotations(nodes, pods, prof, True) == _annotations(nodes, pods, prof, False)


@pytest.mark.parametrize("seed", range(6))
def test_native_serialiser_zoo(built, seed):
    from zoo import zoo
    nodes, pods, prof = zoo(seed, n_pods=60)
    assert _annotations(nodes, pods, prof, True) == _annotations(nodes, pods, prof, False)


def test_go_escaping_of_names(built):
    """Node names / taint values with characters Go escapes, invalid UTF-8."""
    names = ["n<1>", "n&2", "a b", "z\"q\\", "tab\tx", "café"]
    ann = native.Annotator(names, ["P%d" % i for i in range(native.NPLUGINS)], ["cpu", "memory"], [], 
                           __import__("numpy").zeros((0, len(names)), "uint32"))
    import numpy as np
    fs = np.zeros(len(names), np.uint32)
    fs[1] = native.NPLUGINS and 0x1   # rejected by plugin 0 (NodeUnschedulable message)
    f, s, t = ann.annotate([0, 1], [], 0, np.zeros(native.NPLUGINS, np.int64), 1, fs,
                           np.zeros((native.NPLUGINS, len(names)), np.int64),
                           np.zeros((native.NPLUGINS, len(names)), np.int64))
    want = {n: ({"P0": "node(s) were unschedulable"} if i == 1 else {"P0": "passed", "P1": "passed"})
            for i, n in enumerate(names)}
    assert f == A.go_marshal(want)
    assert s == "{}" and t == "{}"


def test_native_serialiser_faster_than_store(built):
    """The point of the row: one call instead of N x (F + 2S) map writes."""
    import binding
    import numpy as np
    nodes, pods, prof = G.config2(n_nodes=2000, n_pods=6, seed=3)
    times = {}
    for nat in (True, False):
        s = F.DebuggableScheduler(nodes, pods, prof, engine=binding.Oracle(4), native_annotations=nat)
        cycs = [s.evaluate(i) for i in range(len(pods))]
        t0 = time.perf_counter()
        for c in cycs:
            s.record(c)
            s.annotations(c.pod)
        times[nat] = time.perf_counter() - t0
    assert times[True] < times[False]


@pytest.mark.parametrize("width", [3, 60])
def test_score_maps_fixed_and_long_keys(built, width):
    """score-result / finalscore-result: plugin keys within and beyond the
    serialiser's fixed-width key slot, values inside and outside its small-
    integer table (negative, 999 / 1000, int64 wrap-around of raw x weight)."""
    import numpy as np
    names = ["n%d" % i for i in range(5)]
    plugins = [("P%d" % i).ljust(width, "x") for i in range(native.NPLUGINS)]
    ann = native.Annotator(names, plugins, ["cpu", "memory"], [], np.zeros((0, len(names)), "uint32"))
    raw = np.zeros((native.NPLUGINS, len(names)), np.int64)
    norm = np.zeros_like(raw)
    raw[0] = [0, 999, 1000, -5, 2 ** 62]
    raw[1] = [7, 100, 12345, 1, 3]
    norm[1] = [100, 0, 55, 999, 1000]
    weight = np.zeros(native.NPLUGINS, np.int64)
    weight[0], weight[1] = 3, 2
    fs = np.zeros(len(names), np.uint32)
    fs[2] = 0x1   # rejected: no score entries
    f, s, t = ann.annotate([0], [1, 0], 1 << 1, weight, 4, fs, raw, norm)

    def wrap(x):
        x &= (1 << 64) - 1
        return x - (1 << 64) if x >> 63 else x
    keep = [i for i in range(len(names)) if fs[i] == 0]
    want_s = {names[i]: {plugins[0]: str(int(raw[0][i])), plugins[1]: str(int(raw[1][i]))} for i in keep}
    want_t = {names[i]: {plugins[0]: str(wrap(int(raw[0][i]) * 3)), plugins[1]: str(wrap(int(norm[1][i]) * 2))}
              for i in keep}
    assert s == A.go_marshal(want_s)
    assert t == A.go_marshal(want_t)
