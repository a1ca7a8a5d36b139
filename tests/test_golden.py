"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py): the
C++ oracle and the Python restatement reproduce them on CPU; the HIP library
reproduces them on the GPU (placements via the batched and the queue paths,
annotation bytes via the DebuggableScheduler mirror)."""
import json
import os

import numpy as np
import pytest

from conftest import pkg
from helpers import pyoracle_annotations, scheduler_annotations

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(HERE, "cases.json")))
KAT = json.load(open(os.path.join(HERE, "readme_kat.json")))

import make_golden_loader as mg  # noqa: E402  (tests/make_golden_loader.py)

E = pkg("encoder")
G = pkg("generator")


@pytest.mark.parametrize("name", sorted(CASES))
def test_inputs_unchanged(name):
    c = CASES[name]
    nodes, pods, prof = mg.make(c["generator"], c["args"])
    assert mg.input_digest(nodes, pods, prof) == c["input_sha256"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_cpp_placements(name):
    import binding
    c = CASES[name]
    nodes, pods, prof = mg.make(c["generator"], c["args"])
    enc = E.Encoder(nodes, pods, prof)
    o = binding.Oracle(2)
    o.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    pl, _ = o.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl, c["placements"])


@pytest.mark.parametrize("name", ["zoo-0", "c2-40x80"])
def test_pyoracle_annotations(name):
    c = CASES[name]
    nodes, pods, prof = mg.make(c["generator"], c["args"])
    anns, _ = pyoracle_annotations(nodes, pods, prof)
    assert [mg.annotation_digest(a) for a in anns] == c["annotations_sha256"]


def test_oracle_cpp_annotations_readme_kat():
    import binding
    nodes, pods, prof = G.readme_kat()
    got = scheduler_annotations(nodes, pods, prof, binding.Oracle(1))
    assert got[0] == KAT


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_golden(built, name):
    native = pkg("native")
    c = CASES[name]
    nodes, pods, prof = mg.make(c["generator"], c["args"])
    enc = E.Encoder(nodes, pods, prof)
    eng = native.Engine(device=0)
    eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    pl, _ = eng.run_queue(0, len(pods))
    np.testing.assert_array_equal(pl, c["placements"])
    anns = scheduler_annotations(nodes, pods, prof, eng)
    assert [mg.annotation_digest(a) for a in anns] == c["annotations_sha256"]


@pytest.mark.gpu
def test_gpu_readme_kat_annotations(built):
    native = pkg("native")
    nodes, pods, prof = G.readme_kat()
    assert scheduler_annotations(nodes, pods, prof, native.Engine(device=0))[0] == KAT
