"""The annotation sidecars of bench.py alone (host serialiser and the device
serialiser, digests): python scripts/annot_bench.py [configs1_pods] [configs2_pods]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PKG = "kube-scheduler-simulator_amd"
native = importlib.import_module(PKG + ".native")
G = importlib.import_module(PKG + ".generator")
E = importlib.import_module(PKG + ".encoder")
B = importlib.import_module(PKG + ".bulk")
n1 = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n3 = int(sys.argv[2]) if len(sys.argv) > 2 else 256
out = {}
nodes, pods, prof = G.config2(n_nodes=5000, n_pods=50000)
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(device=0)
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
out["configs1"] = bench.annotation_sidecar(eng, enc, prof, native, B, n1, 256, 16)
eng.close()
if n3:
    n, p, pr = G.config3(n_nodes=15000, n_pods=n3)
    enc3 = E.Encoder(n, p, pr)
    eng3 = native.Engine(device=0)
    eng3.load(enc3, E.encode_profile(pr, enc3.cluster.res_names))
    out["configs2"] = bench.annotation_sidecar(eng3, enc3, pr, native, B, len(p), 64, 16, label="configs[2]")
    eng3.close()
print(json.dumps(out), flush=True)
