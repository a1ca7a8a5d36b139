"""Golden vector for the ≥30,000-pod configs[2] parity case (VERDICT r3 item
4): the C++ oracle's placements and per-pod results for generator.config3 at
15,000 nodes x 30,000 pods (seed 3), saved as tests/golden/c3_15000x30000.npz.
The oracle takes minutes at this size, so the GPU test compares against this
file instead of re-running it.  Regenerate: python tests/golden/make_c3_large.py [threads]"""
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

N_NODES, N_PODS = 15000, 30000


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    t = time.time()
    nodes, pods, prof = G.config3(n_nodes=N_NODES, n_pods=N_PODS)
    enc = E.Encoder(nodes, pods, prof)
    pf = E.encode_profile(prof, enc.cluster.res_names)
    o = binding.Oracle(threads)
    o.load(enc, pf)
    pl, res = o.run_queue(0, N_PODS)
    np.savez_compressed(os.path.join(HERE, "c3_15000x30000.npz"), placements=np.asarray(pl, np.int32),
                        n_feasible=np.asarray(res["n_feasible"], np.int32),
                        status=np.asarray(res["status"], np.uint32),
                        score_skip=np.asarray(res["score_skip"], np.uint32),
                        pod_count=np.asarray(o.read_state(len(enc.cluster.res_names))[2], np.int32))
    print(f"{N_PODS} pods x {N_NODES} nodes: {int((np.asarray(pl) >= 0).sum())} scheduled, "
          f"{time.time() - t:.0f} s at {threads} threads")


if __name__ == "__main__":
    main()
