"""One process per GPU without an external launcher (bench.py --gpus N).

The driver runs `python bench.py --gpus N` as well as the torchrun form.  When
no launcher set WORLD_SIZE, the parent starts N fresh workers (rank r on
cuda:r) before it touches anything on the GPU itself (no torch, no HIP: an
initialised parent must never fork or exec a GPU process), waits for them and
exits with the first failing worker's status.  Each worker sees the same env
torchrun would give it (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
MASTER_ADDR = 127.0.0.1, MASTER_PORT), so the worker code path is the
torchrun one.  The replicas the ranks run are independent (KEP-184's one
scenario under many schedulers, keps/184-scheduler-simulation/README.md:15-18);
the only exchange is the RCCL gather inside the workers.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Mapping, Optional, Sequence

LAUNCH_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def launched() -> bool:
    """True inside a worker (torchrun's or ours)."""
    return "WORLD_SIZE" in os.environ


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(base: Mapping[str, str], rank: int, world: int, port: int) -> dict:
    """The env of worker `rank`: the parent's env plus torchrun's variables."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def launch(world: int, argv: Sequence[str], env: Optional[Mapping[str, str]] = None,
           timeout: Optional[float] = None, python: str = sys.executable) -> int:
    """Run `python argv...` as `world` ranks; return 0 if every rank exits 0,
    else the first nonzero status (a rank killed by signal s gives 128 + s).
    A failing rank ends the others (they would block in the collective)."""
    base = dict(os.environ if env is None else env)
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        procs.append(subprocess.Popen([python] + list(argv), env=rank_env(base, r, world, port),
                                      start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    try:
        live = set(range(world))
        while live:
            for r in sorted(live):
                s = procs[r].poll()
                if s is None:
                    continue
                live.discard(r)
                if s != 0 and rc == 0:
                    rc = s if s > 0 else 128 - s
                    sys.stderr.write(f"[launcher] rank {r} exited with status {s}; stopping the others\n")
                    _stop(procs, live)
            if timeout is not None and time.monotonic() - t0 > timeout and live:
                sys.stderr.write(f"[launcher] ranks {sorted(live)} still running after {timeout:.0f} s\n")
                _stop(procs, live)
                rc = rc or 124
            time.sleep(0.05)
    finally:
        _stop(procs, {r for r, p in enumerate(procs) if p.poll() is None})
    return rc


def _stop(procs: List[subprocess.Popen], ranks) -> None:
    """SIGTERM each listed rank's own process group, then SIGKILL after 10 s."""
    for r in ranks:
        try:
            os.killpg(procs[r].pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
    t = time.monotonic()
    for r in ranks:
        try:
            procs[r].wait(timeout=max(0.1, 10 - (time.monotonic() - t)))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(procs[r].pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            procs[r].wait()
