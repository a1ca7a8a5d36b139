"""Full-size parity check (checker script, not a product path): run a config's
whole queue on the MI355X through the C ABI and on the CPU oracle, compare
placements, per-pod results and the node state after the queue.

  python scripts/full_parity.py --config 3 [--limit 30000] [--threads 16]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
PKG = "kube-scheduler-simulator_amd"
G = importlib.import_module(PKG + ".generator")
E = importlib.import_module(PKG + ".encoder")
native = importlib.import_module(PKG + ".native")
import binding  # oracle/binding.py: the checker


def replicas(a):
    """Configs 4/5: one GPU replica sweep (ksg_run_replicas) of the first LIMIT
    pods; an evenly spaced subset of the replicas re-run on the oracle."""
    if a.config == 4:
        R = a.replicas or 1024
        nodes, pods, prof, rprofs = G.config4(n_replicas=R)
    else:
        R = a.replicas or 64
        nodes, pods, prof = G.config5(n_pods=a.limit or 500)
        rprofs = [prof] * R   # as scripts/bench_configs.py --config 5
    P = min(a.limit or 500, len(pods))
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    profiles = [E.encode_profile(p, enc.cluster.res_names) for p in rprofs]
    gpu = native.Engine(device=0)
    gpu.load(enc, pf)
    t = time.perf_counter()
    pg, sg = gpu.run_replicas(profiles, 0, P)
    t_gpu = time.perf_counter() - t
    ora = binding.Oracle(nthreads=a.threads)
    ora.load(enc, pf)
    idx = sorted(set(np.linspace(0, R - 1, min(a.check, R)).astype(int).tolist()))
    t = time.perf_counter()
    bad = []
    for k, r in enumerate(idx):
        po, so = ora.run_replicas([profiles[r]], 0, P)
        if not (np.array_equal(pg[r], po[0]) and sg[r].tobytes() == so[0].tobytes()):
            bad.append(r)
        print(f"oracle: replica {r} ({k + 1}/{len(idx)}), {time.perf_counter() - t:.0f}s", file=sys.stderr, flush=True)
    out = {"config": a.config, "nodes": len(nodes), "pods": P, "replicas": R, "checked_replicas": idx,
           "gpu_s": t_gpu, "oracle_s": time.perf_counter() - t, "oracle_threads": a.threads,
           "mismatched_replicas": bad, "placements_and_summaries_equal": not bad}
    print(json.dumps(out), flush=True)
    sys.exit(0 if not bad else 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, choices=(2, 3, 4, 5), default=3)
    ap.add_argument("--replicas", type=int, default=None, help="configs 4/5: replicas on the GPU")
    ap.add_argument("--check", type=int, default=16, help="configs 4/5: replicas re-run on the oracle (evenly spaced)")
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--limit", type=int, default=None, help="compare the first LIMIT pods of the queue")
    a = ap.parse_args()
    if a.config in (4, 5):
        replicas(a)
        return
    make = {2: G.config2, 3: G.config3}[a.config]
    nodes, pods, prof = make(n_pods=a.pods) if a.pods else make()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    P = min(a.limit, len(pods)) if a.limit else len(pods)   # a prefix of the full queue
    gpu = native.Engine(device=0)
    gpu.load(enc, pf)
    t = time.perf_counter()
    pg, rg = gpu.run_queue(0, P)
    t_gpu = time.perf_counter() - t
    ora = binding.Oracle(nthreads=a.threads)
    ora.load(enc, pf)
    t = time.perf_counter()
    parts = []
    for first in range(0, P, a.chunk):   # the oracle's state carries across calls; one progress line per chunk
        parts.append(ora.run_queue(first, min(a.chunk, P - first)))
        print(f"oracle: {first + len(parts[-1][0])}/{P} pods, {time.perf_counter() - t:.0f}s", file=sys.stderr, flush=True)
    po = np.concatenate([x[0] for x in parts])
    ro = {f: np.concatenate([x[1][f] for x in parts]) for f in ("n_feasible", "status", "score_skip")}
    t_cpu = time.perf_counter() - t
    out = {"config": a.config, "nodes": len(nodes), "queue": len(pods), "pods": P, "gpu_s": t_gpu, "oracle_s": t_cpu,
           "oracle_threads": a.threads, "scheduled": int((pg >= 0).sum()),
           "placements_equal": bool(np.array_equal(pg, po)),
           "first_mismatch": int(np.argmax(pg != po)) if not np.array_equal(pg, po) else None}
    for f in ("n_feasible", "status", "score_skip"):
        out[f + "_equal"] = bool(np.array_equal(rg[f], ro[f]))
    R = len(enc.cluster.res_names)
    out["state_equal"] = all(np.array_equal(x, y) for x, y in zip(gpu.read_state(R), ora.read_state(R)))
    print(json.dumps(out), flush=True)
    ok = out["placements_equal"] and out["state_equal"] and all(out[f + "_equal"] for f in ("n_feasible", "status", "score_skip"))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
