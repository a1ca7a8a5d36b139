"""Measure the non-headline configs of BASELINE.json on one MI355X.

  python scripts/bench_configs.py --config 4 [--replicas 1024] [--pods 2000]
  python scripts/bench_configs.py --config 3 [--pods 20000]
  python scripts/bench_configs.py --config 5 [--replicas 64] [--pods 500]

Config 4 / 5 run one what-if replica sweep (ksg_run_replicas: R replicas of
the queue, one workgroup per replica); config 3 runs the single-replica queue
with PodTopologySpread + InterPodAffinity.  Prints one JSON line with pods/s
(replica-pods for sweeps), node-evals/s and the per-kernel roofline from HIP
events on the library's stream.  Pods are a prefix of the config's queue (the
full queue at configs[3]'s 1,024 x 50,000 would run for minutes per sample);
the prefix is stated in the output.  `cpu_baseline`: the C++ restatement
(oracle/, "port") on a bounded sample of the same workload (whole replicas of
the same pod prefix for 4 / 5, a prefix of the queue for 3), at 16 threads and
at every core this process may use, with the CPU model.
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "kube-scheduler-simulator_amd"
G = importlib.import_module(PKG + ".generator")
E = importlib.import_module(PKG + ".encoder")
native = importlib.import_module(PKG + ".native")
metrics = importlib.import_module(PKG + ".metrics")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cores() -> int:
    """Cores this process may actually run on: the affinity mask, capped by the
    cgroup CPU quota and by the CPU share the GPU box exports (it shows the
    whole machine in the mask but grants 16 cores; oversubscribing them
    measures the OS scheduler, not the port)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS", "")   # the GPU box exports its CPU share here
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return n


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(enc, pf, profiles, P: int, threads: int, budget_s: float):
    """Oracle throughput on a bounded sample: replicas one at a time (each the
    full P-pod prefix) for sweeps, 100-pod chunks of the queue otherwise."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding
    o = binding.Oracle(threads)
    o.load(enc, pf)
    N = len(enc.cluster.node_names)
    t0 = time.perf_counter()
    if profiles is not None:
        # replica r's first k pods (each call starts from the loaded state, as
        # every replica does), k doubling from 4 while the budget lasts
        done, r, k = 0, 0, 4
        while time.perf_counter() - t0 < budget_s:
            k = min(k, P)
            o.run_replicas([profiles[r % len(profiles)]], 0, k)
            done += k
            log(f"cpu baseline ({threads} threads): replica {r % len(profiles)}, {k} pods, "
                f"{time.perf_counter() - t0:.1f} s")
            r += 1
            k *= 2
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "replica-pods/s", "cores": threads, "kind": "port",
                "sample": f"{r} replicas, each its first 4, 8, 16 ... pods (at most {P}), {done} replica-pods x "
                          f"{N} nodes ({dt:.1f} s)",
                "node_evals_per_sec": done * N / dt}
    done = 0
    while done < P and time.perf_counter() - t0 < budget_s:
        k = min(100, P - done)
        o.run_queue(done, k, results=False)
        done += k
        log(f"cpu baseline ({threads} threads): {done} pods, {time.perf_counter() - t0:.1f} s")
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "pods/s", "cores": threads, "kind": "port",
            "sample": f"first {done} pods of the queue on the {N}-node cluster ({dt:.1f} s)",
            "node_evals_per_sec": done * N / dt}


def cpu_baselines(enc, pf, profiles, P, budget_s):
    usable = usable_cores()
    out = cpu_baseline(enc, pf, profiles, P, 16, budget_s)
    out.update(cpu_model=cpu_model(), nproc=os.cpu_count(), usable_cores=usable)
    if usable != 16:
        allc = cpu_baseline(enc, pf, profiles, P, usable, budget_s)
        out["all_cores"] = {k: allc[k] for k in ("value", "cores", "sample", "node_evals_per_sec")}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, required=True, choices=(3, 4, 5))
    ap.add_argument("--replicas", type=int, default=None)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--reps", type=int, default=2, help="timed repetitions (after one warmup)")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-kernel HIP-event run (PMC passes)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-placements", default=None, help="write the last run's placements (.npy)")
    ap.add_argument("--pmc", default=None,
                    help="committed PMC summary (profiles/rNN/<name>) whose HBM bytes per dispatch of the "
                         "dominant kernel fill roofline.traffic")
    args = ap.parse_args()

    t0 = time.time()
    profiles = None
    if args.config == 4:
        R = args.replicas or 1024
        P = args.pods or 2000
        nodes, pods, prof, rprofs = G.config4(n_replicas=R, n_nodes=args.nodes or 5000, n_pods=P)
        workload = f"configs[3]: {R} replicas x {len(nodes)} nodes, first {P} pods of the config-2 queue"
    elif args.config == 3:
        P = args.pods or 20000
        nodes, pods, prof = G.config3(n_nodes=args.nodes or 15000, n_pods=P)
        R = 1
        workload = f"configs[2]: {len(nodes)} nodes x {P} pods, PTS + IPA (config3 profile)"
    else:
        R = args.replicas or 64
        P = args.pods or 500
        nodes, pods, prof = G.config5(n_nodes=args.nodes or 100000, n_pods=P)
        rprofs = [prof] * R
        workload = f"configs[4]: {R} replicas x {len(nodes)} nodes, 64 taints/node, 10k images, GPU scalar, {P} pods"
    log(f"generated in {time.time() - t0:.1f}s")
    t0 = time.time()
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    log(f"encoded in {time.time() - t0:.1f}s")
    if args.config in (4, 5):
        profiles = [E.encode_profile(p, enc.cluster.res_names) for p in rprofs]

    eng = native.Engine(device=0)
    eng.load(enc, pf)

    def run():
        if profiles is not None:
            pl, _ = eng.run_replicas(profiles, 0, P)
        else:
            eng.reset_state()
            pl, _ = eng.run_queue(0, P, results=False)
        return pl

    run()   # warmup
    ms = []
    for _ in range(args.reps):
        t = time.perf_counter()
        pl = run()
        ms.append((time.perf_counter() - t) * 1e3)
        log(f"rep: wall {ms[-1]:.1f} ms, device {eng.last_kernel_ms():.1f} ms")
    kms = eng.last_kernel_ms()
    per_eval = metrics.bytes_per_node_eval(enc, prof)
    bpe = sum(per_eval.values())
    roof = None
    if not args.no_timing:
        eng.set_timing(True)
        run()
        ks = eng.kernel_stats()
        eng.set_timing(False)
        roof = metrics.dominant_kernel_roofline(ks, per_eval)
        if roof and args.pmc:
            try:
                tab = json.load(open(os.path.join(ROOT, args.pmc)))
                row = tab.get(roof["kernel"]) or tab.get("ksk::" + roof["kernel"])
            except (OSError, ValueError):
                row = None
            if row and row.get("hbm_bytes_per_dispatch") is not None:
                roof["traffic"] = row["hbm_bytes_per_dispatch"]
                roof["traffic_source"] = args.pmc
                side = roof["traffic"] / (roof["avg_launch_ms"] * 1e-3) / 1e9
                roof["memory_side_GBps"] = side
                roof["memory_side_frac_of_hbm"] = side / roof["peak"]
                roof["traffic_over_algorithmic"] = roof["traffic"] / roof["bytes_per_launch"]
    evals = R * P * len(nodes)
    path, flags = eng.last_run_info()
    out = {
        "config": args.config, "workload": workload, "replicas": R, "nodes": len(nodes), "pods": P,
        "device_ms": kms, "wall_ms": min(ms),
        "pods_per_s": R * P / (kms * 1e-3), "node_evals_per_s": evals / (kms * 1e-3),
        "scheduled": int((pl >= 0).sum()), "bytes_per_node_eval": bpe, "columns": per_eval,
        "roofline": roof,
        "run_path": path, "run_flags": flags,
    }
    if args.config == 3 and flags & native.RUN_TOPO_WINDOW:
        w, d, c = eng.topo_window_stats()
        out["topo_window"] = {"windows": w, "pods_decided": d, "windows_ended_early": c,
                              "mean_pods_per_window": d / max(w, 1)}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baselines(enc, pf, profiles, P, args.cpu_budget)
    if args.save_placements:
        import numpy as np
        np.save(args.save_placements, np.asarray(pl))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
