"""Regenerate the golden vectors in this directory (run from the repo root:
python tests/golden/make_golden.py).

The reference's Go arithmetic cannot run in this image, so
these vectors come from the independent pure-Python restatement
(oracle/pyoracle.py) on the seeded generator workloads; the README KAT part
is checked against the numbers printed in the reference's README.md:56-81 by
tests/test_kat.py.  Each case stores the workload's generator call, a digest
of the encoded inputs (to catch generator drift), the placements, and the
a SHA-256 over every pod's annotations; readme_kat.json stores the
annotation values in full.
"""
import hashlib

import numpy as np
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from conftest import pkg  # noqa: E402
from helpers import pyoracle_annotations  # noqa: E402

G = pkg("generator")
E = pkg("encoder")

CASES = {
    "zoo-0": ("zoo", dict(seed=0, n_pods=40)),
    "zoo-1": ("zoo", dict(seed=1, n_pods=40)),
    "zoo-2": ("zoo", dict(seed=2, n_pods=40)),
    "c1-30x60": ("config1", dict(n_nodes=30, n_pods=60)),
    "c2-40x80": ("config2", dict(n_nodes=40, n_pods=80, seed=21)),
    "c3-24x80": ("config3", dict(n_nodes=24, n_pods=80, apps=6, zones=3)),
}


def make(kind, kw):
    if kind == "zoo":
        from zoo import zoo
        return zoo(**kw)
    return getattr(G, kind)(**kw)


def input_digest(nodes, pods, prof):
    enc = E.Encoder(nodes, pods, prof)
    h = hashlib.sha256()
    for k in sorted(enc.cluster.arrays):
        h.update(k.encode())
        h.update(enc.cluster.arrays[k].tobytes())
    # the pod records as first laid out (144 B; round 5 appended the volume
    # program offset, hashed only when a pod has one), so digests stay put
    pods = enc.workload.pods
    h.update(pods.view(np.uint8).reshape(len(pods), pods.dtype.itemsize)[:, :144].tobytes())
    if (pods["vol"] >= 0).any():
        h.update(pods["vol"].tobytes())
    h.update(enc.workload.prog.tobytes())
    return h.hexdigest()


def annotation_digest(a):
    """SHA-256 (first 32 hex digits) over the pod's annotation key/value pairs, sorted by key."""
    h = hashlib.sha256()
    for k in sorted(a):
        h.update(k.encode() + b"\0" + a[k].encode() + b"\0")
    return h.hexdigest()[:32]


def case_vector(kind, kw):
    nodes, pods, prof = make(kind, kw)
    anns, recs = pyoracle_annotations(nodes, pods, prof)
    names = [n.name for n in nodes]
    return {
        "generator": kind, "args": kw, "input_sha256": input_digest(nodes, pods, prof),
        "placements": [names.index(r["selected"]) if r["selected"] else -1 for r in recs],
        "annotations_sha256": [annotation_digest(a) for a in anns],
    }


def main():
    out = {name: case_vector(kind, kw) for name, (kind, kw) in CASES.items()}
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    nodes, pods, prof = G.readme_kat()
    anns, _ = pyoracle_annotations(nodes, pods, prof)
    with open(os.path.join(HERE, "readme_kat.json"), "w") as f:
        json.dump(anns[0], f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
