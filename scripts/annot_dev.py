"""Device serialiser alone: per-chunk time of the async launch and the wait
(python scripts/annot_dev.py [pods] [chunk] [c1|c3])."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "kube-scheduler-simulator_amd"
native = importlib.import_module(PKG + ".native")
G = importlib.import_module(PKG + ".generator")
E = importlib.import_module(PKG + ".encoder")
B = importlib.import_module(PKG + ".bulk")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cfg = sys.argv[3] if len(sys.argv) > 3 else "c1"
nodes, pods, prof = (G.config3(n_nodes=15000, n_pods=max(n, 1024)) if cfg == "c3"
                     else G.config2(n_nodes=5000, n_pods=50000))
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(device=0)
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
bulk = B.BulkAnnotator(enc, prof, threads=16)
eng.attach_annotator(bulk.annotators[0], bulk.weights, bulk.norm_mask)
for rep in range(3):
    eng.reset_state()
    t0 = time.perf_counter()
    tl, tw = [], []
    tickets = []
    for off in range(0, n, chunk):
        k = min(chunk, n - off)
        t = time.perf_counter()
        _, _, tk = eng.run_queue_json_async(off, k)
        tl.append(time.perf_counter() - t)
        tickets.append((tk, k))
        if len(tickets) >= 2:
            tk0, k0 = tickets.pop(0)
            t = time.perf_counter()
            eng.json_wait(tk0, k0)
            tw.append(time.perf_counter() - t)
    for tk0, k0 in tickets:
        t = time.perf_counter()
        eng.json_wait(tk0, k0)
        tw.append(time.perf_counter() - t)
    wall = time.perf_counter() - t0
    print(f"rep {rep}: {n / wall:.0f} pods/s; launch ms {[round(x * 1e3, 1) for x in tl]}; wait ms {[round(x * 1e3, 1) for x in tw]}",
          flush=True)
eng.reset_state()
eng.set_timing(True)
t = time.perf_counter()
eng.run_queue(0, chunk, capture=native.CaptureBuffers(len(nodes), chunk))
print("capture run (host copies)", round((time.perf_counter() - t) * 1e3, 1), "ms; kernels", eng.kernel_stats())
if os.environ.get("KSG_DUMP_MAPS"):   # diagnosis of exit-time faults: which library sits where
    with open("/proc/self/maps") as f, open(os.environ["KSG_DUMP_MAPS"], "w") as o:
        o.write(f.read())
