"""What-if replica sweep over the GPUs of one node (BASELINE
configs[3] / configs[4]).

Each replica is the same pod queue on the same cluster under its own scheduler
profile (plugin weights, scoring strategy), as the scenario-based-simulation
KEPs describe what-ifs (keps/140-scenario-based-simulation/README.md:62-140).
Replicas are independent, so they are split into contiguous blocks, one block
per rank (one process per GPU); ranks never exchange data while scheduling.
The single collective is the final gather of every replica's placements and
summary to all ranks (RCCL over xGMI on GPUs; gloo in the CPU tests).

The per-pod decision itself is not sharded: every binding changes the node
state the next pod reads.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

SUMMARY_FIELDS = ("scheduled", "unschedulable", "placement_hash", "cpu_requested", "mem_requested")


def shard(n_replicas: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of replicas owned by `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(n_replicas, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _summary_matrix(sums, n: int) -> np.ndarray:
    m = np.zeros((n, len(SUMMARY_FIELDS)), np.int64)
    if sums is not None:
        for k, f in enumerate(SUMMARY_FIELDS):
            m[:, k] = np.asarray(sums[f]).astype(np.uint64).view(np.int64) if f == "placement_hash" \
                else np.asarray(sums[f], np.int64)
    return m


def run_sweep(engine, profiles: Sequence[dict], first: int, count: int, rank: int = 0, world: int = 1,
              device: Optional[str] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Run this rank's block of replicas on `engine`, then gather.

    Returns (placements [R][count] int32, summaries [R][5] int64) on every rank.
    `engine` is native.Engine (the HIP library) in production; any object with
    the same run_replicas() works (the CPU tests pass the oracle).
    `device`: where the gather buffers live ("cuda:<i>" for RCCL, None = CPU/gloo).
    With a process group initialised the gather runs even at world size 1 (the
    bench initialises RCCL at N = 1 too, so the collective executes).
    """
    R = len(profiles)
    lo, hi = shard(R, world, rank)
    mine = list(profiles[lo:hi])
    if mine:
        pl, sums = engine.run_replicas(mine, first, count)
        pl = np.asarray(pl, np.int32)
    else:
        pl, sums = np.zeros((0, count), np.int32), None
    sm = _summary_matrix(sums, len(mine))
    import torch.distributed as dist
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return pl, sm
    import torch
    block = -(-R // world)
    buf = torch.full((block, count + len(SUMMARY_FIELDS) * 2), -1, dtype=torch.int32)
    buf[:len(mine), :count] = torch.from_numpy(pl)
    buf[:len(mine), count:] = torch.from_numpy(sm.view(np.int32).reshape(len(mine), -1))
    if device is not None:
        buf = buf.to(device)
    outs: List = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    all_pl = np.zeros((R, count), np.int32)
    all_sm = np.zeros((R, len(SUMMARY_FIELDS)), np.int64)
    for r, t in enumerate(outs):
        a, b = shard(R, world, r)
        t = t.cpu().numpy()
        all_pl[a:b] = t[:b - a, :count]
        all_sm[a:b] = np.ascontiguousarray(t[:b - a, count:]).view(np.int64)
    return all_pl, all_sm
