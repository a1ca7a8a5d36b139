"""bench.py --gpus N without an external launcher (launcher.py): the parent
starts N ranks with torchrun's env, stays off the GPU, and reports the first
failing rank.  Exercised with a gloo all_gather on CPU (world size 2), the
same wiring the bench's RCCL ranks get on a GPU node."""
import json
import os
import sys

import pytest

from conftest import ROOT, pkg

launcher = pkg("launcher")

RANK_SCRIPT = r"""
import json, os, sys
import torch
import torch.distributed as dist
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
t = torch.tensor([rank * 10 + 1], dtype=torch.int64)
outs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
dist.all_gather(outs, t)
with open(os.path.join(sys.argv[1], f"rank{rank}.json"), "w") as fh:
    json.dump({"rank": rank, "world": world, "local_rank": int(os.environ["LOCAL_RANK"]),
               "gathered": [int(o.item()) for o in outs]}, fh)
dist.barrier()
dist.destroy_process_group()
if len(sys.argv) > 2 and int(sys.argv[2]) == rank:
    sys.exit(3)
"""


def test_rank_env_matches_torchrun():
    env = launcher.rank_env({"PATH": "/bin"}, 1, 4, 29500)
    assert env["RANK"] == env["LOCAL_RANK"] == "1"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"
    assert env["PATH"] == "/bin"
    with pytest.raises(ValueError):
        launcher.rank_env({}, 2, 2, 1)


def test_two_ranks_gather_over_gloo(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = {k: v for k, v in os.environ.items() if k not in launcher.LAUNCH_VARS}
    rc = launcher.launch(2, [str(script), str(tmp_path)], env=env, timeout=120)
    assert rc == 0
    got = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    for r, g in enumerate(got):
        assert (g["rank"], g["world"], g["local_rank"]) == (r, 2, r)
        assert g["gathered"] == [1, 11]


def test_failing_rank_is_reported(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = {k: v for k, v in os.environ.items() if k not in launcher.LAUNCH_VARS}
    assert launcher.launch(2, [str(script), str(tmp_path), "1"], env=env, timeout=120) == 3


def test_bench_refuses_world_mismatch(tmp_path):
    """Under an external launcher, --gpus must equal WORLD_SIZE (the line's
    n_gpus is the ranks that ran)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 rank" in r.stderr
