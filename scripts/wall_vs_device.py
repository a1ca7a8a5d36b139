"""Wall time of one headline step (reset + ksg_run_queue) against the device
time between the library's events, per phase-2 mode (measurement script)."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
native = importlib.import_module("kube-scheduler-simulator_amd.native")

if os.environ.get("WITH_RCCL"):   # the bench's one-rank RCCL group first
    import socket
    import torch
    import torch.distributed as dist
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]), RANK="0", WORLD_SIZE="1")
    sk.close()
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", init_method="env://", world_size=1, rank=0,
                            device_id=torch.device("cuda:0"))
    if os.environ.get("WITH_RCCL") == "2":
        x = torch.zeros(4, device="cuda:0")
        dist.all_reduce(x)
nodes, pods, prof = G.config2()
enc = E.Encoder(nodes, pods, prof)
pf = E.encode_profile(prof, enc.cluster.res_names)
for mode in sys.argv[1:] or ["window", "slot"]:
    os.environ["KSG_BATCH_MODE"] = mode
    eng = native.Engine(device=0)
    eng.load(enc, pf)
    for rep in range(4):
        eng.reset_state()
        t0 = time.perf_counter()
        pl, _ = eng.run_queue(0, len(pods), results=False)
        wall = (time.perf_counter() - t0) * 1e3
        print(f"{mode}: wall {wall:.1f} ms, device {eng.last_kernel_ms():.1f} ms", flush=True)
