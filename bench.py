#!/usr/bin/env python3
"""Headline benchmark: the debuggable scheduler's Filter/Score hot path on MI355X.

Workload (BASELINE.json `metric`: "pods scheduled/sec @5k nodes, default
plugins"): the in-tree default KubeSchedulerConfiguration profile (every
Filter / Score plugin: NodeUnschedulable, NodeName, TaintToleration,
NodeAffinity, NodePorts, NodeResourcesFit, the volume plugins,
PodTopologySpread, InterPodAffinity, BalancedAllocation, ImageLocality) on
5,000 nodes x 50,000 pods, synthetic cluster from generator.config1 (seed 1,
the configs[0] generator at 5,000 nodes: 4 zones, 20 % of the pods with a
zone nodeSelector).  One step = schedule the whole 50,000-pod queue onto the
fresh cluster (reset node state + one ksg_run_queue: filter, score,
normalise, select, assume for every pod, in queue order) with every input
already resident in HBM.

Multi-GPU: the per-pod decision does not shard (every binding changes the
state the next pod reads), so N GPUs run N DISTINCT what-if replicas of the
queue (north star (3)): rank 0 the default profile, rank r >= 1
what-if profile r of generator.default_replica_profiles (every Score weight
in [1, 5], LeastAllocated or MostAllocated), each over the full queue on its
own copy of the cluster (weak scaling: per-GPU work fixed; no data-path
collective).  value = pods scheduled by all ranks / max-over-ranks time; one
RCCL all_gather of every replica's placements per step.  The process group is
RCCL ("nccl") at every N, N = 1 included (a one-rank group on 127.0.0.1), so
the collective runs on the box.

Prints ONE JSON line (rank 0).  The line also carries:
* `configs1`: BASELINE configs[1] (5,000 x 50,000, NodeResourcesFit +
  BalancedAllocation + TaintToleration + NodeAffinity, generator.config2) with
  its own roofline, PMC traffic and CPU baseline (the rounds 1-4 headline);
* `replica_sweep`: BASELINE configs[3], 1,024 what-if replicas (weights and
  strategy per replica) of the first 1,000 pods of configs[1], sharded over
  the N ranks by replicas.run_sweep (contiguous replica blocks, one RCCL
  all_gather of placements + summaries at the end): aggregate
  replica-pods/s over max-over-ranks time, the roofline of its dominant
  kernel, and a digest of all 1,024 replicas' placements (identical at every
  N);
* `cpu_baseline` (rank 0, N = 1): the C++ restatement (oracle/) on a bounded
  prefix of the headline queue, at 16 threads (upstream parallelism) and at
  every host core this process may use, with the CPU model and the limit
  that capped the core count;
* `annotations` / `annotations_configs2` (N = 1): the simulator's product,
  the filter-result / score-result / finalscore-result bytes of the first
  2,000 pods of configs[1] (256 of configs[2]): the device serialiser
  (bulk.annotate_queue_device, values built in HBM and copied to pinned host
  memory) with its digest checked against the host serialiser
  (bulk.annotate_queue, captured rows + ksg_annotate on 16 threads), plus the
  device serialiser's steady state over a longer queue;
* `configs2` (N = 1): BASELINE configs[2], 15,000 nodes x 150,000 pods with
  PodTopologySpread + InterPodAffinity, the whole queue per run on the
  speculative topology queue, placements against the committed golden vector;
* `per_cycle` / `per_cycle_configs2` (N = 1): the drop-in's per-cycle C-ABI
  path, call by call from C (the persistent server, the default since round
  6); `per_cycle_launch` one kernel launch per cycle,
  `per_cycle_hinted` one pending-pod hint per cycle instead of all up front.
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


def usable_cores():
    """(cores, limit): the cores this process may actually run on and what
    capped them -- the affinity mask, the cgroup CPU quota, or the CPU share
    the GPU box exports in OMP_NUM_THREADS (the box shows the whole machine in
    the mask but grants 16 cores)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    limit = "affinity"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max" and int(quota) // int(period) < n:
            n, limit = max(1, int(quota) // int(period)), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and 0 < int(share) < n:
        n, limit = int(share), "OMP_NUM_THREADS"
    return n, limit


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(enc, pf, n_threads: int, budget_s: float, check=None):
    """C++ restatement of the reference algorithm (oracle/, "port"), timed on a
    bounded prefix of the same queue on the same cluster.  With `check` (the
    GPU's placements of the whole queue), the oracle also finishes the queue
    untimed and the line reports whether every placement agrees (VERDICT r5
    item 1: the headline pinned at its own size)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding
    o = binding.Oracle(n_threads)
    o.load(enc, pf)
    n_pods = len(enc.workload.pods)
    done = 0
    chunk = 500
    got = []
    t0 = time.perf_counter()
    while done < n_pods and time.perf_counter() - t0 < budget_s:
        k = min(chunk, n_pods - done)
        got.append(o.run_queue(done, k, results=False)[0])
        done += k
    dt = time.perf_counter() - t0
    out = {"value": done / dt, "unit": "pods/s", "cores": n_threads, "kind": "port",
           "sample": f"first {done} pods of the {n_pods}-pod queue on the same {len(enc.cluster.node_names)}-node "
                     f"cluster ({dt:.1f} s, OpenMP over nodes like the upstream 16-worker Parallelizer)",
           "node_evals_per_sec": done * len(enc.cluster.node_names) / dt}
    if check is not None:
        if done < n_pods:   # the rest of the queue, untimed: the check covers every pod
            got.append(o.run_queue(done, n_pods - done, results=False)[0])
        po = np.concatenate(got)
        bad = np.nonzero(po != np.asarray(check))[0]
        out["placements_checked"] = int(n_pods)
        out["placements_equal_oracle"] = bool(bad.size == 0 and len(check) == n_pods)
        if bad.size:
            out["first_mismatch"] = {"pod": int(bad[0]), "gpu": int(check[bad[0]]), "oracle": int(po[bad[0]]),
                                     "mismatches": int(bad.size)}
    o.close()
    return out


def cpu_baselines(enc, pf, budget_s: float, check=None):
    """BASELINE.md / SURVEY §8(d): 16 threads (upstream parallelism: 16) and
    every host core this process may use (the limit that applied is named);
    when the affinity mask holds more cores than that limit grants, the port
    also runs at min(affinity, 64) threads, labelled as possibly
    oversubscribed (north star: "then all host cores")."""
    usable, limit = usable_cores()
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    out = cpu_baseline(enc, pf, 16, budget_s, check=check)
    out["cpu_model"] = cpu_model()
    out["nproc"] = os.cpu_count()
    out["affinity_cores"] = affinity
    out["usable_cores"] = usable
    out["usable_cores_limit"] = limit
    if usable != 16:
        allc = cpu_baseline(enc, pf, usable, budget_s)
        out["all_cores"] = {k: allc[k] for k in ("value", "cores", "sample", "node_evals_per_sec")}
        out["all_cores"]["limit"] = limit
    wide = min(affinity, 64)
    if affinity > usable and wide > 16:
        w = cpu_baseline(enc, pf, wide, budget_s)
        out["affinity_cores_leg"] = {k: w[k] for k in ("value", "cores", "sample", "node_evals_per_sec")}
        out["affinity_cores_leg"]["note"] = (f"{wide} threads over the {affinity}-core affinity mask; the box "
                                             f"grants {usable} ({limit}): possibly oversubscribed")
    return out


L2_PEAK_GBS = 34500.0   # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md § L2)


def pmc_traffic(kernel, name):
    """HBM bytes per dispatch of `kernel` from a committed PMC summary
    (profiles/run_pmc.sh -> profiles/pmc_summary.py: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), or None."""
    for rnd in ("r6", "r5", "r4", "r3", "r2"):   # the newest round's passes first
        path = os.path.join(ROOT, "profiles", rnd, name)
        try:
            tab = json.load(open(path))
        except (OSError, ValueError):
            continue
        # the summaries key kernels by their demangled name (ksk::ksg_...),
        # the library's timing table by the bare name
        row = (tab.get(kernel) or tab.get("ksk::" + kernel)) if kernel else None
        if row and row.get("hbm_bytes_per_dispatch") is not None:
            return row["hbm_bytes_per_dispatch"], f"profiles/{rnd}/{name}"
    return None, None


def replica_sweep(eng, enc, prof, G, E, metrics, replicas, R: int, P: int, rank: int, world: int, dist, dev):
    """BASELINE configs[3] beside the headline: R what-if replicas (weights and
    strategy per replica, generator.replica_profiles) of the first P pods of
    the same queue on the same cluster, sharded over the ranks by
    replicas.run_sweep (one ksg_run_replicas launch chain per rank, then one
    RCCL all_gather of placements + summaries).  The HBM-bound regime of the
    path: max-over-ranks wall time of the sharded sweep,
    device time of each rank's block from HIP events on the library's
    stream, roofline of the dominant kernel."""
    import hashlib
    import numpy as np
    import torch
    profiles = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(R)]
    replicas.run_sweep(eng, profiles, 0, P, rank=rank, world=world, device=dev)   # warmup
    walls, ms = [], []
    for _ in range(3):
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        pl, sm = replicas.run_sweep(eng, profiles, 0, P, rank=rank, world=world, device=dev)
        torch.cuda.synchronize()
        w = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        walls.append(float(w.item()) * 1e3)
        k = torch.tensor([eng.last_kernel_ms()], dtype=torch.float64, device=dev)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
        ms.append(float(k.item()))
    lo, hi = replicas.shard(R, world, rank)
    ks = []
    if hi > lo:
        eng.set_timing(True)
        eng.run_replicas(profiles[lo:hi], 0, P)
        ks = eng.kernel_stats()
        eng.set_timing(False)
    kms, wms = min(ms), min(walls)
    n = len(enc.cluster.node_names)
    roof = metrics.dominant_kernel_roofline(ks, metrics.bytes_per_node_eval(enc, prof)) if ks else None
    if roof is not None:
        # PMC passes of the same sweep shape at 256 pods per call (64-pod launches, as here)
        roof["traffic"], roof["traffic_source"] = pmc_traffic(roof.get("kernel"), "pmc_config4.json")
        # The narrow replica state (R x N x 16 B = 82 MB at 1,024 x 5,000) stays
        # in the Infinity Cache / L2, so HBM is not the binding ceiling: the
        # algorithmic rate is set beside the aggregate L2 bandwidth
        # (MI355X_MICROARCH.md: 8 x 4 MiB, ~34.5 TB/s) and the memory-side rate
        # (PMC bytes per launch / launch time) beside HBM.
        roof["l2_peak"] = L2_PEAK_GBS
        roof["frac_of_l2"] = roof["achieved"] / L2_PEAK_GBS
        if roof.get("traffic") and roof.get("avg_launch_ms"):
            ms = roof["traffic"] / (roof["avg_launch_ms"] * 1e-3) / 1e9
            roof["memory_side_GBps"] = ms
            roof["memory_side_frac_of_hbm"] = ms / roof["peak"]
        roof["ceiling_note"] = ("replica state resident in L2 / Infinity Cache: bounded by issue, not HBM; "
                                "frac = algorithmic bytes / HBM peak, frac_of_l2 = the same / aggregate L2")
    return {"workload": f"configs[3]: {R} replicas x {n} nodes, first {P} pods of the configs[1] queue, "
                        f"sharded over {world} rank(s), RCCL all_gather of placements + summaries",
            "replica_pods_per_s": R * P / (wms * 1e-3), "node_evals_per_s": R * P * n / (wms * 1e-3),
            "wall_ms": wms, "device_ms_max_rank": kms,
            "device_replica_pods_per_s": R * P / (kms * 1e-3),
            "replicas_per_rank": hi - lo, "collective": "nccl (RCCL) all_gather",
            "placements_sha256": hashlib.sha256(np.ascontiguousarray(pl).tobytes()).hexdigest(),
            "scheduled_total": int(sm[:, 0].sum()),
            "roofline": roof}


def annotation_sidecar(eng, enc, prof, native, B, n_pods: int, chunk: int, threads: int, label: str = "configs[1]"):
    """Annotation bytes for the first n_pods of the queue (bulk.annotate_queue):
    end-to-end wall (device capture + D2H + ksg_annotate on `threads` workers),
    the capture alone, and an xxh3 digest over every pod's three values."""
    import numpy as np
    import xxhash
    digests = np.zeros(n_pods, np.uint64)
    sizes = np.zeros(n_pods, np.int64)

    def sink(i, vals):
        h = xxhash.xxh3_64()
        for v in vals:
            h.update(v)
        digests[i] = h.intdigest()
        sizes[i] = sum(len(v) for v in vals)

    bulk = B.BulkAnnotator(enc, prof, threads=threads)
    dev = None
    try:
        eng.reset_state()
        B.annotate_queue(eng, bulk, 0, min(chunk, n_pods), sink, chunk=chunk)   # warmup
        eng.reset_state()
        t = time.perf_counter()
        pl = B.annotate_queue(eng, bulk, 0, n_pods, sink, chunk=chunk)
        wall = time.perf_counter() - t
        host_digests = digests.copy()
        # The xxh3 sink holds the GIL (python-xxhash does not release it), so
        # it caps either path at ~26 GB/s of hashing; each path is also timed
        # with a light sink (the values' lengths only) for the serialiser's
        # own delivery rate.  Digests come from the xxh3 runs.
        lens = np.zeros(n_pods, np.int64)

        def light(i, vals):
            lens[i] = sum(len(v) for v in vals)

        eng.reset_state()
        t = time.perf_counter()
        B.annotate_queue(eng, bulk, 0, n_pods, light, chunk=chunk)
        wall_light = time.perf_counter() - t
        # the same values serialised on the device (ksg_run_queue_json_async):
        # the capture rows stay in HBM, the finished bytes come back on a copy
        # stream overlapping the next chunk
        try:
            eng.reset_state()
            # warmup over three chunks: the three pinned output buffers (they rotate) get sized
            B.annotate_queue_device(eng, bulk, 0, min(3 * chunk, n_pods), light, chunk=chunk)
            eng.reset_state()
            t = time.perf_counter()
            pl_d = B.annotate_queue_device(eng, bulk, 0, n_pods, light, chunk=chunk)
            wall_dl = time.perf_counter() - t
            eng.reset_state()
            digests[:] = 0
            t = time.perf_counter()
            B.annotate_queue_device(eng, bulk, 0, n_pods, sink, chunk=chunk)
            wall_d = time.perf_counter() - t
            hd = xxhash.xxh3_64()
            hd.update(digests.tobytes())
            dev = {"pods_per_s": n_pods / wall_dl, "wall_s": wall_dl, "annotation_MB_per_s": sizes.sum() / wall_dl / 1e6,
                   "sink": "lengths only (the values delivered to pinned host memory, per-pod views handed out)",
                   "pods_per_s_xxh3_sink": n_pods / wall_d, "digest_xxh3": hd.hexdigest(),
                   "bytes_equal_host": bool((digests == host_digests).all()),
                   "placements_equal_host": bool((pl_d == pl).all()),
                   "path": "ksg_run_queue_json_async (csrc/ksched_json.h) + sink on the annotator's threads"}
        except Exception as e:
            dev = {"error": str(e)}
        digests[:] = host_digests
    finally:
        bulk.close()
    # the captured run alone (device + D2H of the capture arrays), same chunks
    cap = native.CaptureBuffers(len(enc.cluster.node_names), min(chunk, n_pods))
    eng.reset_state()
    eng.set_timing(True)
    t = time.perf_counter()
    dev_ms = 0.0
    ks = {}
    for off in range(0, n_pods, chunk):
        k = min(chunk, n_pods - off)
        eng.run_queue(off, k, capture=cap)
        dev_ms += eng.last_kernel_ms()
        for r in eng.kernel_stats():
            ks[r["name"]] = ks.get(r["name"], 0.0) + r["total_ms"]
    cap_wall = time.perf_counter() - t
    eng.set_timing(False)
    h = xxhash.xxh3_64()
    h.update(digests.tobytes())
    host = {"path": f"device capture + ksg_annotate on {threads} threads (bulk.annotate_queue)",
            "pods_per_s": n_pods / wall, "wall_s": wall, "annotation_MB_per_s": sizes.sum() / wall / 1e6,
            "pods_per_s_light_sink": n_pods / wall_light, "threads": threads}
    ok = isinstance(dev, dict) and "pods_per_s" in dev and dev.get("bytes_equal_host")
    return {"workload": f"{label} cluster, first {n_pods} pods, {chunk}-pod chunks",
            "path": ("device serialiser (bulk.annotate_queue_device): values built in HBM, copied to pinned "
                     "host memory" if ok else "host serialiser (bulk.annotate_queue)"),
            "pods_per_s": dev["pods_per_s"] if ok else n_pods / wall,
            "annotation_bytes": int(sizes.sum()),
            "annotation_MB_per_s": (dev["annotation_MB_per_s"] if ok else sizes.sum() / wall / 1e6),
            "capture_only_pods_per_s": n_pods / cap_wall, "capture_device_ms": dev_ms,
            "capture_kernels_ms": {k: round(v, 3) for k, v in ks.items()},
            "scheduled": int((pl >= 0).sum()), "digest_xxh3": h.hexdigest(),
            "device_serialiser": dev, "host_serialiser": host}


def device_serialiser_long(eng, enc, prof, B, n_pods: int, chunk: int, threads: int):
    """The device serialiser's steady state: ksg_run_queue_json_async over a
    longer queue than the digest sample (pipeline fill and drain amortised),
    light sink; every annotation byte still lands in pinned host memory."""
    import numpy as np
    lens = np.zeros(n_pods, np.int64)

    def light(i, vals):
        lens[i] = sum(len(v) for v in vals)

    bulk = B.BulkAnnotator(enc, prof, threads=threads)
    try:
        eng.reset_state()
        B.annotate_queue_device(eng, bulk, 0, min(3 * chunk, n_pods), light, chunk=chunk)
        eng.reset_state()
        t = time.perf_counter()
        B.annotate_queue_device(eng, bulk, 0, n_pods, light, chunk=chunk)
        wall = time.perf_counter() - t
    finally:
        bulk.close()
    return {"pods": n_pods, "chunk": chunk, "pods_per_s": n_pods / wall, "wall_s": wall,
            "annotation_bytes": int(lens.sum()), "annotation_GB_per_s": lens.sum() / wall / 1e9}


def per_cycle_sidecar(native, G, S, n_nodes: int, warm: int, n_pods: int, make=None, label: str = "configs[1]",
                      server: bool = True, hint_ahead: int = 0):
    """The drop-in's per-cycle path, the calls the Go
    shim makes per scheduling cycle, through the C ABI of libksched.so:
    ksg_snapshot_add_pod -> ksg_snapshot_sync (append to the device
    workload) -> ksg_eval_view (status words + the score rows, left in the
    library's pinned block) ->
    ksg_snapshot_statuses (every rejected node's framework.Status, once per
    pod) -> ksg_snapshot_assume.  configs[1]'s cluster, starting empty; the
    first `warm` pods fill the encoding universe (a pod that adds a label
    value forces a full re-encode, counted), then `n_pods` cycles are timed
    call by call in C (tests/c/cycle_driver.c: no Python in the loop; pod
    views built beforehand).  The placements must equal one ksg_run_queue
    over the same pods."""
    import ctypes as C
    import numpy as np
    nodes, pods, prof = (make or G.config2)(n_nodes=n_nodes, n_pods=warm + n_pods)
    snap = S.Snapshot(prof, nodes)
    # the queue's pending pods are announced up front, as the Go shim's pod
    # informer does (ksg_snapshot_hint_pod): their selectors and templates are
    # in the encoding universe before their cycles, so adding them appends
    # (hint_ahead > 0: only the first warm + hint_ahead up front, then cycle i
    # hints pod i + hint_ahead, as for pods created while the queue runs)
    for p in (pods if hint_ahead <= 0 else pods[:warm + hint_ahead]):
        snap.hint_pod(p)
    prev = os.environ.get("KSG_CYCLE_SERVER")
    os.environ["KSG_CYCLE_SERVER"] = "1" if server else "0"   # read once, when the context opens
    try:
        eng = native.Engine(device=0)
    finally:
        if prev is None:
            os.environ.pop("KSG_CYCLE_SERVER")
        else:
            os.environ["KSG_CYCLE_SERVER"] = prev
    snap.load(eng)
    N = len(nodes)
    rows = native.KsgEvalRows()
    keep = []
    views = []
    for p in pods:
        k = S._Keep()
        views.append(S.pod_view(p, k))
        keep.append(k)
    arr = (S.PodView * len(views))(*views)
    drv = C.CDLL(os.path.join(ROOT, "tests", "c", "libcycle.so"))
    i32p = C.POINTER(C.c_int32)
    drv.cycle_run.restype = C.c_int
    drv.cycle_run.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(S.PodView), C.c_int32, C.c_int32, C.c_void_p,
                              C.c_int32, i32p, C.POINTER(C.c_int64), i32p, i32p, i32p, C.c_int32]
    placed = np.full(warm + n_pods, -1, np.int32)
    phases = np.zeros((n_pods, 5), np.int64)
    ap, rl, where = C.c_int32(), C.c_int32(), C.c_int32(-1)
    rc = drv.cycle_run(snap.h, eng.ctx, arr, len(views), warm, C.addressof(rows), N,
                       placed.ctypes.data_as(i32p), phases.ctypes.data_as(C.POINTER(C.c_int64)),
                       C.byref(ap), C.byref(rl), C.byref(where), hint_ahead)
    if rc != 0:
        raise RuntimeError(f"cycle driver: rc={rc} in phase {where.value}: {snap._err(snap.h).decode()}")
    # the same pods as one device-resident queue
    import importlib
    E = importlib.import_module(PKG + ".encoder")
    enc = E.Encoder(nodes, pods, prof)
    q = native.Engine(device=0)
    q.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    want, _ = q.run_queue(0, len(pods), results=False)
    us = phases / 1e3
    per = us.sum(axis=1)
    names = ["add_pod", "sync", "eval_capture", "statuses", "assume"]
    eval_path = eng.last_run_info()[0]
    eng.close()
    return {"workload": f"{label} cluster ({N} nodes), per-cycle C-ABI path, {n_pods} cycles timed after {warm}",
            "driver": "C (tests/c/cycle_driver.c), CLOCK_MONOTONIC per call",
            "mode": "persistent server (KSG_CYCLE_SERVER=1)" if server else "one launch per cycle",
            "pending_pods_hinted": True if hint_ahead <= 0 else f"one per cycle, {hint_ahead} pods ahead (timed in add_pod)",
            "us_per_cycle_mean": float(per.mean()), "us_per_cycle_p50": float(np.percentile(per, 50)),
            "us_per_cycle_p99": float(np.percentile(per, 99)), "pods_per_s": float(1e6 / per.mean()),
            "breakdown_us_mean": {k: float(us[:, j].mean()) for j, k in enumerate(names)},
            "breakdown_us_p50": {k: float(np.percentile(us[:, j], 50)) for j, k in enumerate(names)},
            "appended": int(ap.value), "full_reloads": int(rl.value),
            "placements_equal_run_queue": bool(np.array_equal(placed, want)),
            "eval_path": eval_path, "eval_path_legend": "5 per-cycle kernel, 6 its topology form"}


def queue_roofline(metrics, kstats, bpe: int, node_evals: int, kms: float, pmc_file: str):
    """The dominant kernel's roofline (algorithmic bytes per launch / its
    average HIP-event duration, SURVEY §8(d) pricing of the node-evals a
    phase-2 launch decides), the whole step beside it, PMC traffic per launch
    from the committed passes and the memory-side rate that traffic implies."""
    roof = metrics.dominant_kernel_roofline(kstats, bpe) if kstats else None
    if roof is None:   # no per-kernel timing: whole step as one launch
        roof = metrics.roofline(bpe, node_evals, kms)
    roof = metrics.price_decided_node_evals(roof, bpe, node_evals)
    roof["step"] = metrics.roofline(bpe, node_evals, kms)
    roof["step"]["kernel_ms"] = kms
    # the timed steps run the persistent walk (one ksg_batch_phase2v_run launch
    # per step, phase 1 / top-k beside it); the per-kernel pass runs with HIP
    # events around every launch, which takes the one-launch-per-batch form of
    # the same walk on one stream
    roof["timing_pass"] = "per-batch launches, one stream (ksg_set_timing); timed steps: persistent walk"
    # HBM bytes per launch of the dominant kernel from the committed PMC passes
    # (profiles/run_pmc.sh -> profiles/pmc_summary.py: 2 x FETCH_SIZE +
    # WRITE_SIZE per dispatch, gfx950-corrected), null when not collected
    roof["traffic"], roof["traffic_source"] = pmc_traffic(roof.get("kernel"), pmc_file)
    if roof.get("traffic") and roof.get("avg_launch_ms"):
        ms = roof["traffic"] / (roof["avg_launch_ms"] * 1e-3) / 1e9
        roof["memory_side_GBps"] = ms
        roof["memory_side_frac_of_hbm"] = ms / roof["peak"]
        roof["traffic_over_algorithmic"] = roof["traffic"] / roof["bytes_per_launch"]
    roof["bytes_per_node_eval"] = bpe
    roof["node_evals_per_step"] = node_evals
    return roof


def configs1_line(native, G, E, metrics, n_nodes: int, n_pods: int, steps: int, cpu_budget: float, local_rank: int):
    """BASELINE configs[1] (generator.config2: NodeResourcesFit LeastAllocated +
    BalancedAllocation + TaintToleration + NodeAffinity) beside the headline:
    pods/s of reset + one ksg_run_queue (best of `steps`), the dominant
    kernel's roofline with its PMC traffic (pmc_config2.json), and the C++
    oracle on a bounded prefix (16 threads).  Returns the line and the loaded
    engine, which the configs[3] / annotation / kubelet legs reuse."""
    nodes, pods, prof = G.config2(n_nodes=n_nodes, n_pods=n_pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng = native.Engine(device=local_rank)
    eng.load(enc, pf)
    best, kms = None, None
    for _ in range(steps + 1):
        eng.reset_state()
        t = time.perf_counter()
        pl, _ = eng.run_queue(0, n_pods, results=False)
        dt = time.perf_counter() - t
        if best is None or dt < best:
            best, kms = dt, eng.last_kernel_ms()
    eng.set_timing(True)
    eng.reset_state()
    eng.run_queue(0, n_pods, results=False)
    ks = eng.kernel_stats()
    eng.set_timing(False)
    bpe = sum(metrics.bytes_per_node_eval(enc, prof).values())
    out = {"workload": f"configs[1]: {n_nodes} nodes x {n_pods} pods, NodeResourcesFit(LeastAllocated)"
                       f"+BalancedAllocation+TaintToleration+NodeAffinity, generator.config2 seed 2",
           "pods_per_s": n_pods / best, "device_pods_per_s": n_pods / (kms * 1e-3),
           "scheduled": int((pl >= 0).sum()),
           "placements_sha256": __import__("hashlib").sha256(pl.tobytes()).hexdigest(),
           "roofline": queue_roofline(metrics, ks, bpe, n_pods * n_nodes, kms, "pmc_config2.json")}
    if cpu_budget > 0:
        out["cpu_baseline"] = cpu_baseline(enc, pf, 16, cpu_budget)
    return out, eng, enc, prof


def kubelet_memory_line(native, G, E, n_nodes: int, n_pods: int, steps: int, configs1_pods_per_s: float):
    """configs[1] with kubelet-style memory (generator.config2_kubelet:
    allocatable a whole number of Ki, not of Mi; 30 % of the pods request
    decimal quantities): the N32 forms do not apply, the speculate-and-verify
    walk runs its wide-memory instance (KSG_RUN_WIDE_MEM).  pods/s of reset +
    one ksg_run_queue (best of `steps`), beside the headline."""
    nodes, pods, prof = G.config2_kubelet(n_nodes=n_nodes, n_pods=n_pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng = native.Engine(device=0)
    eng.load(enc, pf)
    best = None
    for _ in range(steps + 1):
        eng.reset_state()
        t = time.perf_counter()
        pl, _ = eng.run_queue(0, n_pods, results=False)
        dt = time.perf_counter() - t
        best = dt if best is None or dt < best else best
    path, flags = eng.last_run_info()
    v = n_pods / best
    return {"workload": f"configs[1] with kubelet-style memory (generator.config2_kubelet): {n_nodes} nodes x "
                        f"{n_pods} pods", "pods_per_s": v, "configs1_over_this": configs1_pods_per_s / v,
            "wide_memory_walk": bool(flags & native.RUN_WIDE_MEM), "run_flags": flags,
            "scheduled": int((pl >= 0).sum())}


def topo_queue_line(native, G, E, metrics, n_nodes: int, n_pods: int):
    """BASELINE configs[2]: 15,000 nodes x 150,000 pods with PodTopologySpread
    + InterPodAffinity (generator.config3), the whole queue in one
    ksg_run_queue on a fresh cluster (the speculative topology queue,
    ksched_topo_win.h).  A first run with per-kernel timing (the roofline),
    then the timed run; placements against the committed C++-oracle golden
    vector of the same queue when it exists (tests/golden/c3_15000x150000.npz,
    tests/golden/make_golden.py)."""
    import numpy as np
    nodes, pods, prof = G.config3(n_nodes=n_nodes, n_pods=n_pods)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng = native.Engine(device=0)
    eng.load(enc, pf)
    eng.set_timing(True)
    eng.run_queue(0, n_pods, results=False)
    ks = eng.kernel_stats()
    eng.set_timing(False)
    eng.reset_state()
    t = time.perf_counter()
    pl, _ = eng.run_queue(0, n_pods, results=False)
    wall = time.perf_counter() - t
    kms = eng.last_kernel_ms()
    path, flags = eng.last_run_info()
    win = eng.topo_window_stats()
    eng.close()
    per_eval = metrics.bytes_per_node_eval(enc, prof)
    out = {"workload": f"configs[2]: {n_nodes} nodes x {n_pods} pods, PodTopologySpread + InterPodAffinity "
                       "(generator.config3, config3 profile), the whole queue per run",
           "pods_per_s": n_pods / (kms * 1e-3), "pods_per_s_wall": n_pods / wall, "device_ms": kms,
           "scheduled": int((pl >= 0).sum()), "run_flags": flags,
           "speculative_topology_queue": bool(flags & native.RUN_TOPO_WINDOW),
           "windows": {"windows": win[0], "pods_decided": win[1], "ended_early": win[2]},
           "roofline": metrics.dominant_kernel_roofline(ks, per_eval)}
    gold = os.path.join(ROOT, "tests", "golden", f"c3_{n_nodes}x{n_pods}.npz")
    if os.path.exists(gold):
        out["placements_equal_golden"] = bool(np.array_equal(pl, np.load(gold)["placements"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=50000)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=("default", "configs1"), default="default",
                    help="the timed queue: the metric's default profile (headline) or configs[1] (profiling passes)")
    ap.add_argument("--configs1-pods", type=int, default=50000,
                    help="configs[1] line (and the legs on its cluster); 0 disables")
    ap.add_argument("--sweep-replicas", type=int, default=1024, help="configs[3] sidecar; 0 disables")
    ap.add_argument("--sweep-pods", type=int, default=1000)
    ap.add_argument("--annotate-pods", type=int, default=2000, help="annotation sidecar; 0 disables")
    ap.add_argument("--annotate-threads", type=int, default=16)
    ap.add_argument("--annotate-long-pods", type=int, default=8000,
                    help="device serialiser steady state over this many configs[1] pods; 0 disables")
    ap.add_argument("--topo-annotate-long-pods", type=int, default=1024,
                    help="device serialiser steady state over a configs[2] queue of this many pods; 0 disables")
    ap.add_argument("--cycle-pods", type=int, default=2000, help="per-cycle sidecar; 0 disables")
    ap.add_argument("--cycle-warm", type=int, default=500)
    ap.add_argument("--kubelet-pods", type=int, default=50000, help="kubelet-memory line; 0 disables")
    ap.add_argument("--topo-nodes", type=int, default=15000, help="configs[2] cluster of the topology legs")
    ap.add_argument("--topo-cycle-pods", type=int, default=400, help="configs[2] per-cycle leg; 0 disables")
    ap.add_argument("--topo-queue-pods", type=int, default=150000, help="configs[2] full-queue line; 0 disables")
    ap.add_argument("--topo-annotate-pods", type=int, default=256, help="configs[2] annotation leg; 0 disables")
    ap.add_argument("--no-build-check", action="store_true",
                    help="skip the check that libksched.so embeds the tree's source hash")
    args = ap.parse_args()

    # Before anything touches the GPU: the library must be built from this
    # tree's source, and `--gpus N` without a launcher starts N ranks here
    # (launcher.py; the parent stays off the GPU).  Under an outside launcher
    # (torchrun) WORLD_SIZE decides the world and the library is only checked:
    # ranks must not race to rebuild it.
    launcher = importlib.import_module(PKG + ".launcher")
    ge = importlib.import_module("__graft_entry__")
    if not launcher.launched():
        if not args.no_build_check:
            src_hash = ge.ensure_current()
            log(f"libksched.so built from source {src_hash[:12]}")
        if args.gpus > 1:
            sys.exit(launcher.launch(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:] + ["--no-build-check"]))
    elif not args.no_build_check and ge.library_hash() != ge.source_hash():
        raise SystemExit("bench.py: libksched.so does not embed this tree's source hash; run "
                         "__graft_entry__.build() before launching the ranks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s); using {world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist
    if "MASTER_ADDR" not in os.environ:   # N = 1 without a launcher: a one-rank RCCL group
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]), RANK="0",
                          WORLD_SIZE="1", LOCAL_RANK="0")
        sk.close()
    torch.cuda.set_device(local_rank)
    dev = f"cuda:{local_rank}"
    dist.init_process_group(backend="nccl", init_method="env://", world_size=world, rank=rank,
                            device_id=torch.device(dev))
    # one collective before the library opens its streams: RCCL creates its
    # own streams at the first collective, and with GPU_MAX_HW_QUEUES = 4 the
    # order decides which streams share a hardware queue; opened after RCCL's,
    # the library's two streams (phase 2 / phase 1 + top-k) keep separate
    # queues and overlap (127 ms per step instead of 150 ms,
    # scripts/wall_vs_device.py WITH_RCCL=1 / 2)
    warm = torch.zeros(8, device=dev)
    dist.all_reduce(warm)
    torch.cuda.synchronize()

    G = importlib.import_module(PKG + ".generator")
    E = importlib.import_module(PKG + ".encoder")
    native = importlib.import_module(PKG + ".native")
    metrics = importlib.import_module(PKG + ".metrics")
    replicas = importlib.import_module(PKG + ".replicas")

    # ---- the headline: default profile, 5,000 nodes x 50,000 pods ----------------------
    t = time.perf_counter()
    if args.workload == "default":
        nodes, pods, prof = G.config1(n_nodes=args.nodes, n_pods=args.pods)
        whatifs, pmc_file = G.default_replica_profiles, "pmc_default.json"
        label = (f"default profile (every in-tree Filter/Score plugin, weights TaintToleration 3, NodeAffinity 2, "
                 f"PodTopologySpread 2, InterPodAffinity 2, NodeResourcesFit 1 LeastAllocated, BalancedAllocation 1, "
                 f"ImageLocality 1): {len(nodes)} nodes x {len(pods)} pods, generator.config1 seed 1")
    else:   # configs[1] as the timed queue (its PMC passes, profiles/run_pmc.sh)
        nodes, pods, prof = G.config2(n_nodes=args.nodes, n_pods=args.pods)
        whatifs, pmc_file = G.replica_profiles, "pmc_config2.json"
        label = (f"configs[1]: {len(nodes)} nodes x {len(pods)} pods, NodeResourcesFit(LeastAllocated)"
                 f"+BalancedAllocation+TaintToleration+NodeAffinity, generator.config2 seed 2")
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    # this rank's what-if replica: rank 0 the workload's profile, rank r >= 1
    # what-if r of it (distinct weights / strategy)
    prof_r = prof if rank == 0 else whatifs(world)[rank]
    pf_r = pf if rank == 0 else E.encode_profile(prof_r, enc.cluster.res_names)
    log(f"[rank {rank}] encoded {len(nodes)} nodes x {len(pods)} pods in {time.perf_counter() - t:.1f}s")
    eng = native.Engine(device=local_rank)
    eng.load(enc, pf_r)   # inputs resident in HBM from here on
    P = len(pods)

    gather_out = [torch.empty(P, dtype=torch.int32, device=dev) for _ in range(world)]

    def step():
        eng.reset_state()
        pl, _ = eng.run_queue(0, P, results=False)
        # the one exchange of the replica sweep: every replica's placements to every rank (RCCL)
        dist.all_gather(gather_out, torch.from_numpy(pl).to(dev))
        return pl

    for _ in range(args.warmup):
        step()
    kernel_ms = []
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        pl = step()
        kernel_ms.append(eng.last_kernel_ms())
        log(f"[rank {rank}] step wall {(time.perf_counter() - ts) * 1e3:.1f} ms, device {kernel_ms[-1]:.1f} ms")
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    scheduled = int((pl >= 0).sum())
    # every replica's placements, gathered by RCCL in the last step: distinct
    # what-ifs at N > 1 (rank 0's is the default profile's placement)
    import hashlib
    replica_digest = hashlib.sha256(b"".join(g.cpu().numpy().tobytes() for g in gather_out)).hexdigest()
    distinct = len({hashlib.sha256(g.cpu().numpy().tobytes()).hexdigest() for g in gather_out})
    # one extra, untimed step with per-kernel HIP-event timing (ksg_set_timing)
    kstats = []
    try:
        eng.set_timing(True)
        step()
        kstats = eng.kernel_stats()
        eng.set_timing(False)
    except Exception as e:   # timing is diagnostic; never lose the bench line over it
        log(f"[rank {rank}] per-kernel timing unavailable: {e}")

    # ---- configs[1] and the legs on its cluster ----------------------------------------
    c1 = eng1 = enc1 = prof1 = None
    if args.configs1_pods > 0:
        try:
            c1, eng1, enc1, prof1 = configs1_line(native, G, E, metrics, args.nodes, args.configs1_pods, 2,
                                                  0.0 if args.no_cpu_baseline or world > 1 else 8.0, local_rank)
        except Exception as e:
            log(f"[rank {rank}] configs[1] line unavailable: {e}")
    sweep = None
    if args.sweep_replicas > 0 and eng1 is not None:
        try:
            sweep = replica_sweep(eng1, enc1, prof1, G, E, metrics, replicas, args.sweep_replicas,
                                  min(args.sweep_pods, args.configs1_pods), rank, world, dist, dev)
        except Exception as e:   # a sidecar; never lose the headline line over it
            log(f"[rank {rank}] replica sweep unavailable: {e}")
    ann = None
    if world == 1 and args.annotate_pods > 0 and eng1 is not None:
        try:
            B = importlib.import_module(PKG + ".bulk")
            ann = annotation_sidecar(eng1, enc1, prof1, native, B, min(args.annotate_pods, args.configs1_pods), 256,
                                     args.annotate_threads)
            if args.annotate_long_pods > 0 and isinstance(ann.get("device_serialiser"), dict):
                ann["device_serialiser"]["steady_state"] = device_serialiser_long(
                    eng1, enc1, prof1, B, min(args.annotate_long_pods, args.configs1_pods), 256, args.annotate_threads)
        except Exception as e:
            log(f"[rank {rank}] annotation sidecar unavailable: {e}")
    if eng1 is not None:
        eng1.close()
    cyc = cyc_launch = cyc_hint = None
    if world == 1 and args.cycle_pods > 0:
        try:
            S = importlib.import_module(PKG + ".snapshot")
            cyc = per_cycle_sidecar(native, G, S, args.nodes, args.cycle_warm, args.cycle_pods)
            cyc_launch = per_cycle_sidecar(native, G, S, args.nodes, args.cycle_warm, args.cycle_pods, server=False)
            # pods created while the queue runs, one hint per cycle
            cyc_hint = per_cycle_sidecar(native, G, S, args.nodes, args.cycle_warm, args.cycle_pods, hint_ahead=8)
        except Exception as e:
            log(f"[rank {rank}] per-cycle sidecar unavailable: {e}")
    cyc3 = ann3 = None
    if world == 1 and args.topo_cycle_pods > 0:
        try:
            S = importlib.import_module(PKG + ".snapshot")
            cyc3 = per_cycle_sidecar(native, G, S, args.topo_nodes, 300, args.topo_cycle_pods, make=G.config3,
                                     label="configs[2]")
        except Exception as e:
            log(f"[rank {rank}] configs[2] per-cycle sidecar unavailable: {e}")
    if world == 1 and args.topo_annotate_pods > 0:
        try:
            B = importlib.import_module(PKG + ".bulk")
            n3, p3, prof3 = G.config3(n_nodes=args.topo_nodes, n_pods=args.topo_annotate_pods)
            enc3 = E.Encoder(n3, p3, prof3)
            eng3 = native.Engine(device=local_rank)
            eng3.load(enc3, E.encode_profile(prof3, enc3.cluster.res_names))
            ann3 = annotation_sidecar(eng3, enc3, prof3, native, B, len(p3), 64, args.annotate_threads,
                                      label="configs[2]")
            eng3.close()
            if args.topo_annotate_long_pods > 0 and isinstance(ann3.get("device_serialiser"), dict):
                n3, p3, prof3 = G.config3(n_nodes=args.topo_nodes, n_pods=args.topo_annotate_long_pods)
                enc3 = E.Encoder(n3, p3, prof3)
                eng3 = native.Engine(device=local_rank)
                eng3.load(enc3, E.encode_profile(prof3, enc3.cluster.res_names))
                ann3["device_serialiser"]["steady_state"] = device_serialiser_long(
                    eng3, enc3, prof3, B, len(p3), 64, args.annotate_threads)
                eng3.close()
        except Exception as e:
            log(f"[rank {rank}] configs[2] annotation sidecar unavailable: {e}")
    topo = None
    if world == 1 and args.topo_queue_pods > 0:
        try:
            topo = topo_queue_line(native, G, E, metrics, args.topo_nodes, args.topo_queue_pods)
        except Exception as e:
            log(f"[rank {rank}] configs[2] queue line unavailable: {e}")
    kub = None
    if world == 1 and args.kubelet_pods > 0 and c1 is not None:
        try:
            kub = kubelet_memory_line(native, G, E, args.nodes, min(args.kubelet_pods, args.pods), 2,
                                      c1["pods_per_s"])
        except Exception as e:
            log(f"[rank {rank}] kubelet-memory line unavailable: {e}")

    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        pods_per_s = world * P * args.steps / elapsed
        node_evals = world * P * len(nodes) * args.steps / elapsed
        bpe = sum(metrics.bytes_per_node_eval(enc, prof).values())
        kms = float(np.mean(kernel_ms))
        try:
            roof = queue_roofline(metrics, kstats, bpe, P * len(nodes), kms, pmc_file)
        except Exception as e:
            log(f"per-kernel roofline unavailable: {e}")
            roof = metrics.roofline(bpe, P * len(nodes), kms)
        out = {
            "metric": "pods scheduled/sec @5k nodes, default plugins; node-evals/sec; % HBM peak",
            "value": pods_per_s, "unit": "pods/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": label + (f"; ranks 1..{world - 1}: distinct what-if profiles"
                                            if world > 1 else ""),
                       "nodes": len(nodes), "pods": P, "parallelism": f"replicas{world}",
                       "pods_scheduled_per_step": scheduled, "distinct_replica_placements": distinct,
                       "replica_placements_sha256": replica_digest},
            "node_evals_per_sec": node_evals,
            "roofline": roof,
        }
        out["source_hash"] = {"library": ge.library_hash(), "tree": ge.source_hash()}
        out["source_hash"]["matches"] = out["source_hash"]["library"] == out["source_hash"]["tree"]
        for key, val in (("configs1", c1), ("replica_sweep", sweep), ("annotations", ann), ("per_cycle", cyc),
                         ("per_cycle_launch", cyc_launch), ("per_cycle_hinted", cyc_hint),
                         ("kubelet_memory", kub), ("configs2", topo), ("per_cycle_configs2", cyc3),
                         ("annotations_configs2", ann3)):
            if val is not None:
                out[key] = val
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baselines(enc, pf, args.cpu_budget, check=pl)
            # the headline's placements against the oracle over the whole queue
            out["placements_equal_oracle"] = out["cpu_baseline"].get("placements_equal_oracle")
        print(json.dumps(out), flush=True)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
