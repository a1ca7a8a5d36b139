"""Replica sweep: sharding arithmetic, and the N>1 path with
world_size-2 gloo process groups on CPU.  The engine in these tests is the
C++ oracle (test infrastructure); on the GPU the same run_sweep() drives the
HIP library and gathers over RCCL (tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest

from conftest import pkg

G = pkg("generator")
E = pkg("encoder")
replicas = pkg("replicas")


@pytest.mark.parametrize("R,world", [(1, 1), (6, 2), (7, 2), (1024, 8), (3, 8), (64, 8)])
def test_shard_covers_every_replica_once(R, world):
    seen = []
    for r in range(world):
        lo, hi = replicas.shard(R, world, r)
        assert 0 <= lo <= hi <= R
        assert hi - lo in (R // world, -(-R // world))
        seen.extend(range(lo, hi))
    assert seen == list(range(R))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload():
    nodes, pods, base = G.config2(n_nodes=80, n_pods=120, seed=7)
    enc = E.Encoder(nodes, pods, base)
    profs = [E.encode_profile(p, enc.cluster.res_names) for p in G.replica_profiles(5)]
    return enc, profs


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist
    import binding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    enc, profs = _workload()
    o = binding.Oracle(1)
    o.load(enc, profs[0])
    pl, sm = replicas.run_sweep(o, profs, 0, len(enc.workload.pods), rank=rank, world=world)
    np.save(os.path.join(out_dir, f"pl{rank}.npy"), pl)
    np.save(os.path.join(out_dir, f"sm{rank}.npy"), sm)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_gather_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    import binding
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    enc, profs = _workload()
    o = binding.Oracle(1)
    o.load(enc, profs[0])
    want_pl, want_sm = replicas.run_sweep(o, profs, 0, len(enc.workload.pods))
    assert want_pl.shape == (5, 120)
    assert (want_sm[:, 0] + want_sm[:, 1] == 120).all()
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"pl{r}.npy"), want_pl)
        np.testing.assert_array_equal(np.load(tmp_path / f"sm{r}.npy"), want_sm)
    # replicas differ in weights/strategy, so their placements are not all equal
    assert len({want_pl[r].tobytes() for r in range(5)}) > 1
