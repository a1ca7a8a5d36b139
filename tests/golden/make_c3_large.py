"""Golden vectors for the large configs[2] parity cases (VERDICT r3 item 4,
r4 item 4): the C++ oracle's placements and per-pod results for
generator.config3 at 15,000 nodes x P pods (seed 3), saved as
tests/golden/c3_15000x<P>.npz (P = 30,000, and the full 150,000-pod queue).
The oracle takes minutes to hours at these sizes, so the GPU tests compare
against these files instead of re-running it.
Regenerate: python tests/golden/make_c3_large.py [threads] [pods]"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import importlib  # noqa: E402

G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
import binding  # noqa: E402

N_NODES = 15000


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    N_PODS = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
    t = time.time()
    nodes, pods, prof = G.config3(n_nodes=N_NODES, n_pods=N_PODS)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    o = binding.Oracle(threads)
    o.load(enc, pf)
    chunks, step = [], 2000
    for lo in range(0, N_PODS, step):   # in chunks, with progress (the full queue runs for a long time)
        chunks.append(o.run_queue(lo, min(step, N_PODS - lo)))
        print(f"  {lo + len(chunks[-1][0])} pods, {time.time() - t:.0f} s", flush=True)
    pl = np.concatenate([c[0] for c in chunks])
    res = {k: np.concatenate([np.asarray(c[1][k]) for c in chunks]) for k in ("n_feasible", "status", "score_skip")}
    np.savez_compressed(os.path.join(HERE, f"c3_15000x{N_PODS}.npz"), placements=np.asarray(pl, np.int32),
                        n_feasible=np.asarray(res["n_feasible"], np.int32),
                        status=np.asarray(res["status"], np.uint32),
                        score_skip=np.asarray(res["score_skip"], np.uint32),
                        pod_count=np.asarray(o.read_state(len(enc.cluster.res_names))[2], np.int32))
    print(f"{N_PODS} pods x {N_NODES} nodes: {int((np.asarray(pl) >= 0).sum())} scheduled, "
          f"{time.time() - t:.0f} s at {threads} threads")


if __name__ == "__main__":
    main()
