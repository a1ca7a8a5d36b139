"""Diagnostic: phase-2 segment shares from the KSG_STAMPS build (never the
measured library).  Run on the GPU box: python profiles/stamps.py"""
import ctypes as C
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
native = importlib.import_module("kube-scheduler-simulator_amd.native")

n_pods = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
# argv[2] "default": the headline's default profile (generator.config1 at 5,000 nodes)
if len(sys.argv) > 2 and sys.argv[2] == "default":
    nodes, pods, prof = G.config1(n_nodes=5000, n_pods=n_pods)
else:
    nodes, pods, prof = G.config2(n_pods=n_pods)
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(lib_path=os.path.join(ROOT, "kube-scheduler-simulator_amd", "libksched_stamps.so"))
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
eng.run_queue(0, n_pods, results=False)
ms = eng.last_kernel_ms()
st = (C.c_ulonglong * 16)()
fn = eng.lib.ksg_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
assert fn(eng.ctx, st) == 0
tot = sum(st[1:])
mode = os.environ.get("KSG_BATCH_MODE", "pipe")
if mode == "pipe":
    names = ["(unused)", "bu + candidate buffer reads", "evaluate pod j+1 (both versions)",
             "candidates of pod j+1 + loads", "fold + decide", "contributions (reductions)",
             "results (lane 0)", "assume + record rotation", "candidate stores (wait for loads)", "barrier"]
    print(f"[pipe] {n_pods} pods, kernel {ms:.1f} ms, {ms * 1e3 / n_pods:.2f} us/pod (stamped build)")
    tot = sum(st[1:10])
    for i in range(1, 10):
        print(f"  {names[i]:36s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / tot:5.1f} %")
    sys.exit(0)
if mode == "tcol":
    names = ["(loop top)", "rescan check + P1 reads", "decide", "assume + result", "next-pod candidate + loads",
             "row read", "column eval + running maxima"]
    print(f"[tcol] {n_pods} pods, kernel {ms:.1f} ms, {ms * 1e3 / n_pods:.2f} us/pod (stamped build)")
    tot = sum(st[0:7])
    for i in range(0, 7):
        print(f"  {names[i]:36s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / tot:5.1f} %")
    sys.exit(0)
if mode == "spec":
    names = ["setup (LDS staging, initial pointers)", "S: speculate + publish (wave 0)", "V: wave 0 verifying after S",
             "barrier (other waves still verifying)", "A: aggregate + barrier", "C: check + commit (wave 0)",
             "barrier", "epilogue"]
    print(f"[spec] {n_pods} pods, kernel {ms:.1f} ms, {ms * 1e3 / n_pods:.2f} us/pod (stamped build); "
          f"rounds per batch {st[15] / max(1, (n_pods + 63) // 64):.2f}, speculation steps per batch "
          f"{st[14] / max(1, (n_pods + 63) // 64):.1f} in {st[12] / max(1, (n_pods + 63) // 64):.1f} macro-steps, "
          f"step-on iterations per batch {st[13] / max(1, (n_pods + 63) // 64):.1f}")
    names += ["setup: wait for phase 1 / top-k", "setup: staging (pods, programs, T)"]
    names[0] = "setup: carried slots, pod records, initial pointers"
    tot = sum(st[0:10])
    for i in (8, 9, 0, 1, 2, 3, 4, 5, 6, 7):
        print(f"  {names[i]:40s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / tot:5.1f} %")
    sys.exit(0)
if mode in ("slot", "window"):
    names = ["(start)", "X: speculate + issue next-pod loads", "X: changed node + DPP reductions",
             "Y: barrier 1 + decide (+renorm)", "Y: row update + results", "barrier 2",
             "Y: next-pod records + top set (waits)", "Y: fetched column decode"]
else:
    names = ["(start)", "A: changed nodes + top sets", "barrier 1", "B: decide (+rescan)",
             "B: next-pod LDS writes", "barrier 2 (waits for the assume)"]
print(f"[{mode}] {n_pods} pods, kernel {ms:.1f} ms, {ms * 1e3 / n_pods:.2f} us/pod (stamped build)")
if mode in ("slot", "window") and any(st[8:13]):   # the finer split of segments 1 and 2 (loop order)
    names += [""] * 8
    names[8], names[9], names[1] = "X0: pod setup (LDS pod/P1 reads)", "X1: speculated node (top set, C)", "X2: issue next-pod loads"
    names[10], names[11], names[12] = "X3a: to slot evaluation", "X3b: slot read + Fit/BA scores", "X3c: normalise + key"
    names[2] = "X3d: DPP reductions + partials"
    for i in (8, 9, 1, 10, 11, 12, 2, 3, 6, 7, 4, 5):
        print(f"  {names[i]:36s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / tot:5.1f} %")
    sys.exit(0)
for i in range(1, 8 if mode in ("slot", "window") else 6):
    print(f"  {names[i]:36s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / tot:5.1f} %")
