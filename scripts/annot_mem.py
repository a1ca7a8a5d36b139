"""CPU read speed of the device serialiser's output buffer (pinned) vs a copy."""
import importlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import xxhash
PKG = "kube-scheduler-simulator_amd"
native = importlib.import_module(PKG + ".native")
G = importlib.import_module(PKG + ".generator")
E = importlib.import_module(PKG + ".encoder")
B = importlib.import_module(PKG + ".bulk")
nodes, pods, prof = G.config2(n_nodes=5000, n_pods=50000)
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(device=0)
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
bulk = B.BulkAnnotator(enc, prof, threads=16)
eng.attach_annotator(bulk.annotators[0], bulk.weights, bulk.norm_mask)
pl, _, js, offs = eng.run_queue_json(0, 256)
n = len(js)
for rep in range(2):
    t = time.perf_counter(); h = xxhash.xxh3_64(); h.update(js); a = time.perf_counter() - t
    t = time.perf_counter(); arr = np.frombuffer(js, np.uint8).copy(); b = time.perf_counter() - t
    t = time.perf_counter(); h = xxhash.xxh3_64(); h.update(arr); c = time.perf_counter() - t
    print(f"{n/1e6:.0f} MB: xxh3 on pinned {n/a/1e9:.1f} GB/s, copy out {n/b/1e9:.1f} GB/s, xxh3 on copy {n/c/1e9:.1f} GB/s", flush=True)
