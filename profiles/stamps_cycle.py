"""Per-cycle kernel segment stamps (diagnostic KSG_STAMPS build, never the
measured library): python profiles/stamps_cycle.py [n_nodes] [pods]

ksg_eval of configs[1]'s pods one by one (eval + commit from Python), then the
per-segment s_memtime sums of workgroup 0 of ksg_eval_cycle (ksched_cycle.h
KSG_YSTAMP slots 0-6) divided by the evaluations."""
import ctypes as C, importlib, os, sys, time
ROOT = os.getcwd(); sys.path.insert(0, ROOT)
G = importlib.import_module("kube-scheduler-simulator_amd.generator")
E = importlib.import_module("kube-scheduler-simulator_amd.encoder")
native = importlib.import_module("kube-scheduler-simulator_amd.native")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
nodes, pods, prof = G.config2(n_nodes=N, n_pods=P)
enc = E.Encoder(nodes, pods, prof)
eng = native.Engine(lib_path=os.path.join(ROOT, "kube-scheduler-simulator_amd", "libksched_stamps.so"))
eng.load(enc, E.encode_profile(prof, enc.cluster.res_names))
for i in range(50):
    r = eng.eval(i)
fn = eng.lib.ksg_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
st0 = (C.c_ulonglong * 16)(); fn(eng.ctx, st0)
t = time.perf_counter()
for i in range(50, P):
    r = eng.eval(i)
    if r.selected >= 0:
        eng.commit(i, r.selected)
dt = (time.perf_counter() - t) / (P - 50)
st = (C.c_ulonglong * 16)(); fn(eng.ctx, st)
names = ["entry (arguments, columns, programs)", "evaluate (filters, scores)", "reductions, slots, status+raw rows",
         "exchange wait (folding the lines)", "(fold: empty since r5)", "norm+total rows + release", "record + done word"]
d = [st[i] - st0[i] for i in range(7)]
tot = sum(d)
print(f"[cycle] {N} nodes, {P-50} evals, {dt*1e6:.1f} us per eval+commit (python loop)")
for i, nm in enumerate(names):
    print(f"  {nm:34s} {d[i] / (P-50):8.0f} clk  {100 * d[i] / max(tot,1):5.1f} %")
print(f"  total {tot/(P-50):.0f} clk (s_memtime, workgroup 0)")
fe = eng.lib.ksg_debug_eval_stamps
fe.argtypes = [C.c_void_p, C.c_void_p]
es = (C.c_ulonglong * 16)()
if fe(eng.ctx, es) == 0:
    PL = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
          "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread", "(other)"]
    labels = ["prefilter/node_set + loop entry"] + [f"filter {x}" for x in PL] + ["scores Fit+BA", "scores Image+Taint", "score NodeAffinity"]
    tot = sum(es)
    print(f"[eval_node_src] lane 0 of workgroup 0, all calls since load ({tot} clk)")
    for i in range(16):
        if es[i]:
            print(f"  {labels[i]:34s} {es[i] / (P):8.0f} clk/eval  {100 * es[i] / max(tot,1):5.1f} %")
