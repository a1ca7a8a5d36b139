"""Phase-2 variants of the batched config-2 path side by side on one MI355X
(measurement script): pods/s of a full queue (HIP events on the library's
stream) and per-kernel launch times (ksg_set_timing, serialised) per
KSG_BATCH_MODE / KSG_PIPE_WINDOW / KSG_SLOT_BLOCK setting.

  python scripts/compare_modes.py [--pods 50000] [--nodes 5000]
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
native = importlib.import_module("kube-scheduler-simulator_amd.native")

MODES = [("spec", {"KSG_BATCH_MODE": "spec"}),
         ("window", {"KSG_BATCH_MODE": "window"}),
         ("slot", {"KSG_BATCH_MODE": "slot"}), ("slot-128", {"KSG_BATCH_MODE": "slot", "KSG_SLOT_BLOCK": "128"})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--modes", default=",".join(m for m, _ in MODES))
    a = ap.parse_args()
    nodes, pods, prof = G.config2(n_nodes=a.nodes, n_pods=a.pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    keys = ("KSG_BATCH_MODE", "KSG_PIPE_WINDOW", "KSG_SLOT_BLOCK")
    want = set(a.modes.split(","))
    ref = None
    for name, env in MODES:
        if name not in want:
            continue
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = native.Engine(device=0)
        for k in keys:
            os.environ.pop(k, None)
        eng.load(enc, pf)
        eng.run_queue(0, len(pods), results=False)   # warm-up
        best = None
        for _ in range(3):
            eng.reset_state()
            pl, _ = eng.run_queue(0, len(pods), results=False)
            ms = eng.last_kernel_ms()
            best = ms if best is None else min(best, ms)
        if ref is None:
            ref = pl
        eng.reset_state()
        eng.set_timing(True)
        eng.run_queue(0, len(pods), results=False)
        ks = eng.kernel_stats()
        print(json.dumps({"mode": name, "pods_per_s": len(pods) / (best * 1e-3), "device_ms": best,
                          "same_placements": bool((pl == ref).all()),
                          "kernels_us": {k["name"]: round(k["avg_ms"] * 1e3, 2) for k in ks}}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
