#!/usr/bin/env python3
"""Headline benchmark: the debuggable scheduler's Filter/Score hot path on MI355X.

Workload (BASELINE.json configs[1]): 5,000 nodes x 50,000 pods, NodeResourcesFit
(LeastAllocated) + BalancedAllocation + TaintToleration + NodeAffinity (+ the
always-on NodeUnschedulable / NodeName filters), synthetic cluster from
generator.config2 (seed 2).  One step = schedule the whole 50,000-pod queue
onto the fresh cluster (reset node state + one ksg_run_queue launch: filter,
score, normalise, select, assume for every pod, in queue order) with every
input already resident in HBM.

Multi-GPU: the per-pod decision does not shard (every binding changes the
state the next pod reads), so N GPUs run N independent what-if replicas of the
same queue (weak scaling, no data-path collective); value = pods scheduled by
all ranks / max-over-ranks time.

Prints ONE JSON line (rank 0).  At N=1 the line also carries
`replica_sweep`: BASELINE configs[3] (1,024 what-if replicas of the first
1,000 pods on the same cluster), the HBM-bound regime of the same path, with
the roofline of its dominant kernel.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "kube-scheduler-simulator_amd"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(enc, pf, n_threads: int, budget_s: float):
    """C++ restatement of the reference algorithm (oracle/, "port"), timed on a
    bounded prefix of the same queue on the same cluster."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding
    o = binding.Oracle(n_threads)
    o.load(enc, pf)
    n_pods = len(enc.workload.pods)
    done = 0
    chunk = 500
    t0 = time.perf_counter()
    while done < n_pods and time.perf_counter() - t0 < budget_s:
        k = min(chunk, n_pods - done)
        o.run_queue(done, k, results=False)
        done += k
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "pods/s", "cores": n_threads, "kind": "port",
            "sample": f"first {done} pods of the {n_pods}-pod queue on the same {len(enc.cluster.node_names)}-node "
                      f"cluster ({dt:.1f} s, OpenMP over nodes like the upstream 16-worker Parallelizer)",
            "node_evals_per_sec": done * len(enc.cluster.node_names) / dt}


def replica_sweep(eng, enc, prof, G, E, metrics, R: int, P: int):
    """BASELINE configs[3] beside the headline: R what-if replicas (weights and
    strategy per replica, generator.replica_profiles) of the first P pods of
    the same queue on the same cluster, one ksg_run_replicas launch chain.
    This is the HBM-bound regime of the path; device time from
    HIP events on the library's stream, roofline of the dominant kernel."""
    profiles = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(R)]
    eng.run_replicas(profiles, 0, P)   # warmup
    ms, walls = [], []
    for _ in range(3):
        t = time.perf_counter()
        eng.run_replicas(profiles, 0, P)
        walls.append((time.perf_counter() - t) * 1e3)
        ms.append(eng.last_kernel_ms())
    eng.set_timing(True)
    eng.run_replicas(profiles, 0, P)
    ks = eng.kernel_stats()
    eng.set_timing(False)
    kms = min(ms)
    n = len(enc.cluster.node_names)
    return {"workload": f"configs[3]: {R} replicas x {n} nodes, first {P} pods of the configs[1] queue",
            "replica_pods_per_s": R * P / (kms * 1e-3), "node_evals_per_s": R * P * n / (kms * 1e-3),
            "device_ms": kms, "wall_ms": min(walls),
            "roofline": metrics.dominant_kernel_roofline(ks, metrics.bytes_per_node_eval(enc, prof))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep-replicas", type=int, default=1024, help="configs[3] sidecar; 0 disables")
    ap.add_argument("--sweep-pods", type=int, default=1000)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl", init_method="env://")

    G = importlib.import_module(PKG + ".generator")
    E = importlib.import_module(PKG + ".encoder")
    native = importlib.import_module(PKG + ".native")
    metrics = importlib.import_module(PKG + ".metrics")

    t = time.perf_counter()
    nodes, pods, prof = G.config2(n_nodes=args.nodes, n_pods=args.pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    log(f"[rank {rank}] encoded {len(nodes)} nodes x {len(pods)} pods in {time.perf_counter() - t:.1f}s")
    eng = native.Engine(device=local_rank)
    eng.load(enc, pf)   # inputs resident in HBM from here on
    P = len(pods)

    gather_out = None
    if dist:
        gather_out = [torch.empty(P, dtype=torch.int32, device=f"cuda:{local_rank}") for _ in range(world)]

    def step():
        eng.reset_state()
        pl, _ = eng.run_queue(0, P, results=False)
        if dist:
            # the one exchange of the replica sweep: every replica's placements to every rank (RCCL)
            dist.all_gather(gather_out, torch.from_numpy(pl).to(f"cuda:{local_rank}"))
        return pl

    for _ in range(args.warmup):
        step()
    kernel_ms = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pl = step()
        kernel_ms.append(eng.last_kernel_ms())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    scheduled = int((pl >= 0).sum())
    # one extra, untimed step with per-kernel HIP-event timing (ksg_set_timing)
    kstats = []
    try:
        eng.set_timing(True)
        step()
        kstats = eng.kernel_stats()
        eng.set_timing(False)
    except Exception as e:   # timing is diagnostic; never lose the bench line over it
        log(f"[rank {rank}] per-kernel timing unavailable: {e}")

    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        pods_per_s = world * P * args.steps / elapsed
        node_evals = world * P * len(nodes) * args.steps / elapsed
        per_eval = metrics.bytes_per_node_eval(enc, prof)
        bpe = sum(per_eval.values())
        kms = float(np.mean(kernel_ms))
        try:
            roof = metrics.dominant_kernel_roofline(kstats, bpe)
        except Exception as e:
            log(f"per-kernel roofline unavailable: {e}")
            roof = None
        if roof is None:   # no per-kernel timing: whole step as one launch
            roof = metrics.roofline(bpe, P * len(nodes), kms)
        roof["step"] = metrics.roofline(bpe, P * len(nodes), kms)
        roof["step"]["kernel_ms"] = kms
        # HBM bytes per launch of the dominant kernel from the committed PMC
        # passes (profiles/run_pmc.sh -> profiles/pmc_summary.py: 2 x FETCH_SIZE
        # + WRITE_SIZE per dispatch, gfx950-corrected), null when not collected
        roof["traffic"] = None
        pmc = os.path.join(ROOT, "profiles", "r1", "pmc_config2.json")
        if os.path.exists(pmc) and roof.get("kernel"):
            try:
                row = json.load(open(pmc)).get(roof["kernel"])
                if row:
                    roof["traffic"] = row["hbm_bytes_per_dispatch"]
                    roof["traffic_source"] = "profiles/r1/pmc_config2.json"
            except Exception:
                pass
        roof["bytes_per_node_eval"] = bpe
        roof["node_evals_per_launch"] = P * len(nodes)
        out = {
            "metric": "pods scheduled/sec @5k nodes, default plugins; node-evals/sec; % HBM peak",
            "value": pods_per_s, "unit": "pods/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": f"configs[1]: {len(nodes)} nodes x {P} pods, NodeResourcesFit(LeastAllocated)"
                                   f"+BalancedAllocation+TaintToleration+NodeAffinity, generator.config2 seed 2",
                       "nodes": len(nodes), "pods": P, "parallelism": f"replicas{world}",
                       "pods_scheduled_per_step": scheduled},
            "node_evals_per_sec": node_evals,
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(enc, pf, args.cpu_threads, args.cpu_budget)
        if args.sweep_replicas > 0 and world == 1:
            try:
                out["replica_sweep"] = replica_sweep(eng, enc, prof, G, E, metrics, args.sweep_replicas,
                                                     min(args.sweep_pods, P))
            except Exception as e:   # a sidecar; never lose the headline line over it
                log(f"replica sweep unavailable: {e}")
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
