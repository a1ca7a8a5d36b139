"""Diagnostic: per-pod segment shares of the chip-wide topology path
(ksg_topo_coop) from the KSG_STAMPS build, workgroup 0's clock (never the
measured library).  Run on the GPU box: python profiles/stamps_topo.py [pods]"""
import ctypes as C
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
native = importlib.import_module("kube-scheduler-simulator_amd.native")

n_pods = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
nodes, pods, prof = G.config3(n_pods=n_pods)
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(lib_path=os.path.join(ROOT, "kube-scheduler-simulator_amd", "libksched_stamps.so"))
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
if len(sys.argv) > 2 and sys.argv[2] == "eval":
    # the per-cycle form: one ksg_eval_view (the topology kernel on one pod,
    # reading the per-cycle domain tables) and one ksg_commit per pod, after
    # n_pods // 2 queued pods
    warm = n_pods // 2
    eng.run_queue(0, warm, results=False)
    st0 = (C.c_ulonglong * 16)()
    f0 = eng.lib.ksg_debug_stamps
    f0.argtypes = [C.c_void_p, C.c_void_p]
    assert f0(eng.ctx, st0) == 0
    import time
    t = time.perf_counter()
    for j in range(warm, n_pods):
        # ksg_eval_view (capture mode 2, the per-cycle tables), rows left in the library
        r, v = native.KsgResult(), native.KsgEvalRows()
        eng._check(eng._eval_view(eng.ctx, j, C.byref(r), C.byref(v)))
        if r.selected >= 0:
            eng.commit(j, r.selected)
    ms = (time.perf_counter() - t) * 1e3
    n_pods = n_pods - warm
else:
    st0 = None
    eng.run_queue(0, n_pods, results=False)
    ms = eng.last_kernel_ms()
st = (C.c_ulonglong * 16)()
fn = eng.lib.ksg_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
assert fn(eng.ctx, st) == 0
if st0 is not None:   # the per-cycle calls only
    for i in range(16):
        st[i] -= st0[i]
tot = sum(st)
win = bool(eng.last_run_info()[1] & native.RUN_TOPO_WINDOW)
names = ["setup (stage pod, layout)", "phase 1: merge / publish", "barrier 1", "2a: merged counts to LDS",
         "2b: reset next set, IPA skips", "2c3: sweep A, IPA score", "2d: reductions, marks", "barrier 2",
         "3c: normalise, argmax", "barrier 3", "phase 4 (select, assume)", "2c1: sweep A, load + filters",
         "2c2: sweep A, PTS soft", "3a: fold phase-2 partials", "3b: marks, sizes, weights", "phase 1: node loop"]
if win:   # the speculative topology queue: a row ends after 3c (ksched_topo_win.h)
    names[8] = "3c: normalise (static totals)"
    names[9] = "window: tile lists, facts, row arrival"
    names[10] = "window: launch arrival + walk (wg 0)"
order = [0, 15, 1, 2, 3, 4, 11, 12, 5, 6, 7, 13, 14, 8, 9, 10]
print(f"[topo coop{' window rows' if win else ''}] {n_pods} pods x {len(nodes)} nodes, kernel {ms:.1f} ms, {ms * 1e3 / n_pods:.2f} us/pod (stamped)")
for i in order:
    print(f"  {names[i]:34s} {st[i] / n_pods:10.0f} cycles/pod  {100 * st[i] / max(tot, 1):5.1f} %")
