"""ctypes binding of the C ABI in include/ksched.h (libksched.so).

The shared library is built in-tree by `__graft_entry__.build()` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library cannot be loaded
the import of `Lib` fails loudly, so no GPU test can pass on a CPU path.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import shutil
import weakref
from typing import Optional

import numpy as np

# Kernel arguments in device memory: the batched walk launches one
# single-workgroup kernel per 64-pod batch, and fetching each launch's
# argument block from host memory cost 8-16 % of the headline
# (scripts/gpu_kernarg_ab.sh).  The HIP runtime reads it at its first call;
# a caller's own setting wins (libksched.so sets the same default at load).
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from . import encoder as E

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libksched.so")

NPLUGINS = 14
PL_TAINT_TOLERATION, PL_NODE_AFFINITY = 2, 3   # KSG_PL_* of include/ksched.h
MAX_RES = 8
MAX_SHAPE = 16     # KSG_MAX_SHAPE

# Every live native handle (Engine, Snapshot, Annotator) is closed by an
# atexit hook before the interpreter tears down, most recently opened first,
# so no context is freed from __del__ during finalisation or left for the HIP
# runtime's own exit handlers (under rocprofv3 the process used to end in
# SIGSEGV inside exit()).  KSG_EXIT_MAPS=<path> also copies
# /proc/self/maps there at that point, to map a crash in a later exit handler
# to its library.
_LIVE: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()
_SEQ = [0]
_HOOKED = [False]


def _close_all():
    path = os.environ.get("KSG_EXIT_MAPS")
    if path:
        try:
            shutil.copyfile("/proc/self/maps", path)
        except OSError:
            pass
    if os.environ.get("KSG_NO_EXIT_CLOSE") == "1":   # diagnostic: leave the handles to finalisation
        return
    for k in sorted(_LIVE.keys(), reverse=True):
        obj = _LIVE.get(k)
        if obj is not None:
            try:
                obj.close()
            except Exception:
                pass


def track(obj) -> None:
    """Register a native handle for the exit hook (registered on the first
    handle, i.e. after the process has initialised the GPU: atexit runs the
    newest hooks first, so this one runs before torch's)."""
    _SEQ[0] += 1
    _LIVE[_SEQ[0]] = obj
    if not _HOOKED[0]:
        atexit.register(_close_all)
        _HOOKED[0] = True


i32p = C.POINTER(C.c_int32)
u32p = C.POINTER(C.c_uint32)
i64p = C.POINTER(C.c_int64)
u8p = C.POINTER(C.c_uint8)
f64p = C.POINTER(C.c_double)


class KsgNodes(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("n_res", C.c_int32), ("alloc", i64p), ("requested", i64p),
                ("nonzero", i64p), ("allowed_pods", i32p), ("pod_count", i32p), ("unschedulable", u8p),
                ("n_label_cols", C.c_int32), ("label_val", u32p), ("label_num", i64p), ("label_num_ok", u8p),
                ("max_taints", C.c_int32), ("taints", u32p), ("n_taint_vocab", C.c_int32), ("taint_effect", u8p),
                ("max_images", C.c_int32), ("images", u32p), ("n_images", C.c_int32),
                ("n_port_vocab", C.c_int32)]


class KsgTopology(C.Structure):
    _fields_ = [("n_selectors", C.c_int32), ("n_templates", C.c_int32), ("tmpl_col", i32p),
                ("tmpl_kind", i32p), ("tmpl_weight", i32p), ("col_vocab", i32p), ("col_unique", u8p),
                ("log_table", f64p), ("log_n", C.c_int32)]


class KsgWorkload(C.Structure):
    _fields_ = [("pods", C.c_void_p), ("n_pods", C.c_int32), ("prog", i32p), ("prog_len", C.c_int64)]


class KsgProfile(C.Structure):
    _fields_ = [("n_filter", C.c_int32), ("filter_order", C.c_int32 * NPLUGINS), ("score_mask", C.c_uint32),
                ("weight", C.c_int32 * NPLUGINS), ("fit_strategy", C.c_int32), ("fit_n", C.c_int32),
                ("fit_res", C.c_int32 * MAX_RES), ("fit_w", C.c_int64 * MAX_RES), ("ba_n", C.c_int32),
                ("ba_res", C.c_int32 * MAX_RES), ("hard_pod_affinity_weight", C.c_int32),
                ("flags", C.c_uint32), ("fit_ignored_res", C.c_uint32), ("shape_n", C.c_int32),
                ("shape_util", C.c_int32 * MAX_SHAPE), ("shape_score", C.c_int32 * MAX_SHAPE), ("pad", C.c_int32)]


class KsgResult(C.Structure):
    _fields_ = [("selected", C.c_int32), ("n_feasible", C.c_int32), ("status", C.c_uint32),
                ("score_skip", C.c_uint32)]


RESULT_DTYPE = np.dtype([("selected", "<i4"), ("n_feasible", "<i4"), ("status", "<u4"), ("score_skip", "<u4")])


class KsgCapture(C.Structure):
    _fields_ = [("fstatus", u32p), ("raw", i64p), ("norm", i64p), ("total", i64p)]


class KsgEvalRows(C.Structure):
    """ksg_eval_rows: the per-cycle rows in library memory."""
    _fields_ = [("n_nodes", C.c_int32), ("elem_bytes", C.c_int32), ("fstatus", u32p),
                ("raw", C.c_void_p * NPLUGINS), ("norm", C.c_void_p * NPLUGINS), ("total", C.c_void_p),
                ("norm_from_raw", C.c_uint32), ("norm_scored", C.c_uint32), ("norm_max", C.c_int64 * NPLUGINS)]


def derive_norm(plugin: int, raw: np.ndarray, mx: int, fstatus: np.ndarray, scored: bool) -> np.ndarray:
    """DefaultNormalizeScore of a row the per-cycle kernel leaves to the host
    (ksg_eval_rows.norm_from_raw): TaintToleration reversed, NodeAffinity
    plain, integer division by the maximum over the feasible nodes; 0 at
    infeasible nodes and when the pod was not scored."""
    out = np.zeros(len(raw), np.int64)
    if not scored:
        return out
    feas = fstatus == 0
    r = raw.astype(np.int64)
    if plugin == PL_TAINT_TOLERATION:
        v = 100 - (100 * r) // mx if mx else np.full(len(r), 100, np.int64)
    else:
        v = (100 * r) // mx if mx else r
    out[feas] = v[feas]
    return out


class KsgNodeState(C.Structure):
    _fields_ = [("requested", i64p), ("nonzero", i64p), ("pod_count", i32p)]


class KsgReplicaSummary(C.Structure):
    _fields_ = [("scheduled", C.c_int32), ("unschedulable", C.c_int32), ("placement_hash", C.c_uint64),
                ("cpu_requested", C.c_int64), ("mem_requested", C.c_int64)]


SUMMARY_DTYPE = np.dtype([("scheduled", "<i4"), ("unschedulable", "<i4"), ("placement_hash", "<u8"),
                          ("cpu_requested", "<i8"), ("mem_requested", "<i8")])
assert SUMMARY_DTYPE.itemsize == C.sizeof(KsgReplicaSummary)

ST_SCORED = 1
ST_IPA_PREFILTER_SKIP = 2
ST_IPA_PRESCORE_SKIP = 4
ST_SCORE_ERROR = 8


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


class Marshalled:
    """Keeps the numpy buffers behind the C structs alive."""

    def __init__(self, enc: "E.Encoder"):
        ec = enc.cluster
        a = ec.arrays
        self.keep = {}

        def keep(name, arr, dtype):
            arr = np.ascontiguousarray(arr, dtype=dtype)
            self.keep[name] = arr
            return arr

        N = len(ec.node_names)
        self.n_nodes = N
        self.nodes = KsgNodes(
            n_nodes=N, n_res=len(ec.res_names),
            alloc=_ptr(keep("alloc", a["alloc"], np.int64), i64p),
            requested=_ptr(keep("requested", a["requested"], np.int64), i64p),
            nonzero=_ptr(keep("nonzero", a["nonzero"], np.int64), i64p),
            allowed_pods=_ptr(keep("allowed", a["allowed_pods"], np.int32), i32p),
            pod_count=_ptr(keep("pod_count", a["pod_count"], np.int32), i32p),
            unschedulable=_ptr(keep("unsched", a["unschedulable"], np.uint8), u8p),
            n_label_cols=len(ec.label_cols),
            label_val=_ptr(keep("label_val", a["label_val"], np.uint32), u32p),
            label_num=_ptr(keep("label_num", a["label_num"], np.int64), i64p),
            label_num_ok=_ptr(keep("label_num_ok", a["label_num_ok"], np.uint8), u8p),
            max_taints=ec.max_taints, taints=_ptr(keep("taints", a["taints"], np.uint32), u32p),
            n_taint_vocab=len(ec.taint_vocab),
            taint_effect=_ptr(keep("taint_effect", a["taint_effect"], np.uint8), u8p),
            max_images=ec.max_images, images=_ptr(keep("images", a["images"], np.uint32), u32p),
            n_images=ec.n_images, n_port_vocab=getattr(ec, "n_port_vocab", 0))
        self.topo = KsgTopology(
            n_selectors=ec.n_selectors, n_templates=ec.n_templates,
            tmpl_col=_ptr(keep("tmpl_col", a["tmpl_col"], np.int32), i32p),
            tmpl_kind=_ptr(keep("tmpl_kind", a["tmpl_kind"], np.int32), i32p),
            tmpl_weight=_ptr(keep("tmpl_weight", a["tmpl_weight"], np.int32), i32p),
            col_vocab=_ptr(keep("col_vocab", a["col_vocab"], np.int32), i32p),
            col_unique=_ptr(keep("col_unique", a["col_unique"], np.uint8), u8p),
            log_table=_ptr(keep("log_table", a["log_table"], np.float64), f64p),
            log_n=int(len(a["log_table"])))
        wl = enc.workload
        pods = keep("pods", wl.pods, E.POD_DTYPE)
        prog = keep("prog", wl.prog, np.int32)
        self.n_pods = len(pods)
        self.workload = KsgWorkload(pods=pods.ctypes.data, n_pods=len(pods),
                                    prog=_ptr(prog, i32p), prog_len=len(prog))


def make_profile(fields: dict) -> KsgProfile:
    p = KsgProfile()
    for k, v in fields.items():
        attr = getattr(p, k)
        if isinstance(v, (list, tuple)):
            for i, x in enumerate(v):
                attr[i] = x
        else:
            setattr(p, k, v)
    return p


RUN_NARROW_SWEEP, RUN_SLOT32, RUN_SPEC, RUN_WIDE_MEM, RUN_TOPO_WINDOW = 1, 2, 8, 16, 32   # ksg_last_run_info flags


class CaptureBuffers:
    """Host buffers for `count` pods of capture output."""

    def __init__(self, n_nodes: int, count: int = 1):
        self.fstatus = np.zeros((count, n_nodes), np.uint32)
        self.raw = np.zeros((count, NPLUGINS, n_nodes), np.int64)
        self.norm = np.zeros((count, NPLUGINS, n_nodes), np.int64)
        self.total = np.zeros((count, n_nodes), np.int64)
        self.struct = KsgCapture(_ptr(self.fstatus, u32p), _ptr(self.raw, i64p), _ptr(self.norm, i64p),
                                 _ptr(self.total, i64p))


def _bind(lib, prefix: str):
    def f(name, restype, *argtypes):
        fn = getattr(lib, prefix + name)
        fn.restype = restype
        fn.argtypes = list(argtypes)
        return fn
    return f


class KsgKernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("kind", C.c_int32), ("calls", C.c_int32), ("total_ms", C.c_double),
                ("units", C.c_double)]


class KschedError(RuntimeError):
    pass


class Engine:
    """One evaluator context (ksg_ctx) behind the C ABI."""

    PREFIX = "ksg_"

    def __init__(self, lib_path: Optional[str] = None, device: int = 0):
        path = lib_path or LIB_PATH
        if not os.path.exists(path):
            raise KschedError(f"{path} not found: run __graft_entry__.build() (no CPU fallback exists)")
        self.lib = C.CDLL(path)
        self._declare()
        self.ctx = C.c_void_p()
        self._check(self._open(device, C.byref(self.ctx)))
        self._m: Optional[Marshalled] = None
        self._nn = 0
        track(self)

    def _declare(self):
        f = _bind(self.lib, self.PREFIX)
        vp = C.c_void_p
        self._open = f("open", C.c_int, C.c_int, C.POINTER(C.c_void_p))
        self._close = f("close", C.c_int, vp)
        self._err = f("last_error", C.c_char_p, vp)
        self._set_profile = f("set_profile", C.c_int, vp, C.POINTER(KsgProfile))
        self._load_nodes = f("load_nodes", C.c_int, vp, C.POINTER(KsgNodes), C.POINTER(KsgTopology))
        self._load_workload = f("load_workload", C.c_int, vp, C.POINTER(KsgWorkload))
        self._eval = f("eval", C.c_int, vp, C.c_int32, C.POINTER(KsgResult), C.POINTER(KsgCapture))
        # the product library's zero-copy per-cycle call (the CPU oracle has none)
        self._eval_view = (f("eval_view", C.c_int, vp, C.c_int32, C.POINTER(KsgResult), C.POINTER(KsgEvalRows))
                           if hasattr(self.lib, self.PREFIX + "eval_view") else None)
        self._commit = f("commit", C.c_int, vp, C.c_int32, C.c_int32)
        self._run_queue = f("run_queue", C.c_int, vp, C.c_int32, C.c_int32, i32p, vp, C.POINTER(KsgCapture))
        # the product library's device annotation serialiser (the CPU oracle has none)
        self._attach = self._run_queue_json = self._run_queue_json_async = self._json_wait = None
        if hasattr(self.lib, self.PREFIX + "annotator_attach"):
            self._attach = f("annotator_attach", C.c_int, vp, vp, C.POINTER(C.c_int64), C.c_uint32)
            self._run_queue_json = f("run_queue_json", C.c_int, vp, C.c_int32, C.c_int32, i32p, vp,
                                     C.POINTER(C.c_void_p), C.POINTER(C.POINTER(C.c_int64)))
            self._run_queue_json_async = f("run_queue_json_async", C.c_int, vp, C.c_int32, C.c_int32, i32p, vp,
                                           C.POINTER(C.c_int32))
            self._json_wait = f("json_wait", C.c_int, vp, C.c_int32, C.POINTER(C.c_void_p),
                                C.POINTER(C.POINTER(C.c_int64)))
        self._read_state = f("read_state", C.c_int, vp, C.POINTER(KsgNodeState))
        self._reset_state = f("reset_state", C.c_int, vp)
        self._uncommit = f("uncommit", C.c_int, vp, C.c_int32, C.c_int32)
        self._preempt = f("preempt_victims", C.c_int, vp, C.c_int32, i32p, C.c_int32, i32p, i32p, i32p,
                          C.POINTER(C.c_uint8))
        self._eval_skipping = f("eval_skipping", C.c_int, vp, C.c_int32, C.c_uint32, C.POINTER(KsgResult),
                                C.POINTER(KsgCapture))
        self._append = f("append_pods", C.c_int, vp, C.POINTER(KsgWorkload), C.c_int64)
        self._declare_extra(f)

    def _declare_extra(self, f):
        vp = C.c_void_p
        self._run_replicas = f("run_replicas", C.c_int, vp, C.POINTER(KsgProfile), C.c_int32, C.c_int32,
                               C.c_int32, i32p, vp)
        self._eval_pod = f("eval_pod", C.c_int, vp, vp, i32p, C.c_int64, C.POINTER(KsgResult),
                           C.POINTER(KsgCapture))
        self._last_ms = f("last_kernel_ms", C.c_int, vp, C.POINTER(C.c_double))
        self._run_info = f("last_run_info", C.c_int, vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32))
        self._recoveries = f("recoveries", C.c_int, vp, C.POINTER(C.c_int32))
        self._win_stats = f("topo_window_stats", C.c_int, vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                            C.POINTER(C.c_int64))
        self._set_timing = f("set_timing", C.c_int, vp, C.c_int)
        self._kernel_stats = f("kernel_stats", C.c_int, vp, C.POINTER(KsgKernelStat), C.c_int32,
                               C.POINTER(C.c_int32))
        self.abi_version = f("abi_version", C.c_int)()

    def _check(self, rc: int):
        if rc != 0:
            msg = self._err(self.ctx).decode() if self.ctx else ""
            raise KschedError(f"{self.PREFIX} call failed rc={rc}: {msg}")

    def close(self):
        if self.ctx:
            self._close(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- loading --------------------------------------------------------
    def load(self, enc: "E.Encoder", prof_fields: dict):
        self._m = Marshalled(enc)
        self.set_profile(prof_fields)
        self._check(self._load_nodes(self.ctx, C.byref(self._m.nodes), C.byref(self._m.topo)))
        self._check(self._load_workload(self.ctx, C.byref(self._m.workload)))

    def set_profile(self, prof_fields: dict):
        self._check(self._set_profile(self.ctx, C.byref(make_profile(prof_fields))))
        self.profile_fields = prof_fields

    def _snapshot_loaded(self, snap):
        """Loaded through the native snapshot encoder (snapshot.Snapshot)."""
        n = C.c_int32()
        snap.lib.ksg_snapshot_counts(snap.h, C.byref(n), None, None, None)
        self._m = None
        self._nn = n.value

    @property
    def n_nodes(self) -> int:
        return self._m.n_nodes if self._m is not None else self._nn

    # -- evaluation -----------------------------------------------------
    def eval(self, pod: int, capture: Optional[CaptureBuffers] = None) -> KsgResult:
        r = KsgResult()
        self._check(self._eval(self.ctx, pod, C.byref(r), C.byref(capture.struct) if capture else None))
        return r

    def eval_skipping(self, pod: int, filter_skip: int, capture: Optional[CaptureBuffers] = None) -> KsgResult:
        """ksg_eval_skipping: ksg_eval with the Filter plugins in the
        `filter_skip` bit mask skipped (DefaultPreemption's node-static verdict)."""
        r = KsgResult()
        self._check(self._eval_skipping(self.ctx, pod, filter_skip, C.byref(r),
                                        C.byref(capture.struct) if capture else None))
        return r

    def eval_view(self, pod: int):
        """ksg_eval_view: (result, {"fstatus": u32[N], "raw"/"norm": {plugin: int64[N]}, "total": int64[N]}),
        copied out of the library's rows (valid there until the next evaluation)."""
        r, v = KsgResult(), KsgEvalRows()
        self._check(self._eval_view(self.ctx, pod, C.byref(r), C.byref(v)))
        n = v.n_nodes
        ct = {1: C.c_uint8, 2: C.c_int16, 4: C.c_int32, 8: C.c_int64}[v.elem_bytes]

        def row(ptr):
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), (n,)).astype(np.int64)
        fs = np.ctypeslib.as_array(v.fstatus, (n,)).copy()
        raw = {p: row(v.raw[p]) for p in range(NPLUGINS) if v.raw[p]}
        norm = {p: row(v.norm[p]) for p in range(NPLUGINS) if v.norm[p]}
        for p in range(NPLUGINS):   # the rows the caller derives (ksg_eval_rows.norm_from_raw)
            if (v.norm_from_raw >> p) & 1:
                norm[p] = derive_norm(p, raw[p], v.norm_max[p], fs, (v.norm_scored >> p) & 1)
        out = {"fstatus": fs, "elem_bytes": v.elem_bytes, "raw": raw, "norm": norm,
               "total": row(v.total) if v.total else None}
        return r, out

    def append_pods(self, pods: np.ndarray, prog: np.ndarray, prog_base: int):
        """ksg_append_pods: pods (POD_DTYPE, absolute program offsets) whose
        programs are pool words [prog_base, prog_base + len(prog))."""
        pods = np.ascontiguousarray(pods, E.POD_DTYPE)
        prog = np.ascontiguousarray(prog, np.int32)
        wl = KsgWorkload(pods=pods.ctypes.data, n_pods=len(pods), prog=_ptr(prog, i32p), prog_len=len(prog))
        self._check(self._append(self.ctx, C.byref(wl), prog_base))

    def eval_pod(self, pod: np.ndarray, prog: np.ndarray, capture: Optional[CaptureBuffers] = None) -> KsgResult:
        """ksg_eval_pod: an encoded pod outside the workload (offsets into prog)."""
        rec = np.ascontiguousarray(np.asarray(pod, E.POD_DTYPE).reshape(1))
        prog = np.ascontiguousarray(prog, np.int32)
        r = KsgResult()
        self._check(self._eval_pod(self.ctx, rec.ctypes.data, _ptr(prog, i32p), len(prog), C.byref(r),
                                   C.byref(capture.struct) if capture else None))
        return r

    def commit(self, pod: int, node: int):
        self._check(self._commit(self.ctx, pod, node))

    def commit_batch(self, pods, nodes):
        """ksg_commit_batch: NodeInfo.AddPod of pods[i] onto nodes[i], one launch
        (the snapshot's replay of its bindings)."""
        pods = np.ascontiguousarray(pods, np.int32)
        nodes = np.ascontiguousarray(nodes, np.int32)
        fn = getattr(self.lib, self.PREFIX + "commit_batch")
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, i32p, i32p, C.c_int32]
        self._check(fn(self.ctx, _ptr(pods, i32p), _ptr(nodes, i32p), len(pods)))

    def uncommit(self, pod: int, node: int):
        """A preemption victim's deletion (ksg_uncommit: NodeInfo.RemovePod)."""
        self._check(self._uncommit(self.ctx, pod, node))

    def preempt_victims(self, pod: int, cand_nodes, vic_off, vic_pod):
        """SelectVictimsOnNode for every candidate node (ksg_preempt_victims).
        Returns (fits[n_cand] bool, victim[len(vic_pod)] bool)."""
        cand = np.ascontiguousarray(cand_nodes, np.int32)
        off = np.ascontiguousarray(vic_off, np.int32)
        vic = np.ascontiguousarray(vic_pod, np.int32)
        if len(off) != len(cand) + 1:
            raise ValueError("vic_off needs n_cand + 1 entries")
        fits = np.zeros(len(cand), np.int32)
        victim = np.zeros(max(len(vic), 1), np.uint8)
        self._check(self._preempt(self.ctx, pod, _ptr(cand, i32p), len(cand), _ptr(off, i32p), _ptr(vic, i32p),
                                  _ptr(fits, i32p), victim.ctypes.data_as(C.POINTER(C.c_uint8))))
        return fits.astype(bool), victim[:len(vic)].astype(bool)

    def run_queue(self, first: int, count: int, capture: Optional[CaptureBuffers] = None,
                  results: bool = True):
        pl = np.zeros(count, np.int32)
        res = np.zeros(count, RESULT_DTYPE) if results else None
        self._check(self._run_queue(self.ctx, first, count, _ptr(pl, i32p),
                                    res.ctypes.data if res is not None else None,
                                    C.byref(capture.struct) if capture else None))
        return pl, res

    def attach_annotator(self, ann: "Annotator", weight, normalize_mask: int):
        """ksg_annotator_attach: the annotator's escaped pieces to the device,
        with the Store's score weights [NPLUGINS] (for run_queue_json)."""
        if self._attach is None:
            raise KschedError(f"{self.PREFIX}annotator_attach: this library has no device serialiser")
        w = np.ascontiguousarray(weight, np.int64)
        self._check(self._attach(self.ctx, ann.h, w.ctypes.data_as(C.POINTER(C.c_int64)), int(normalize_mask)))

    def run_queue_json(self, first: int, count: int):
        """ksg_run_queue_json: placements, results, the three annotation
        values of every pod serialised on the device (one read-only
        memoryview over the context's pinned buffer, valid until the next
        call) and their offsets [3 * count + 1] (pod k's values at
        offsets[3k : 3k + 4])."""
        pl = np.zeros(count, np.int32)
        res = np.zeros(count, RESULT_DTYPE)
        js = C.c_void_p()
        off = C.POINTER(C.c_int64)()
        self._check(self._run_queue_json(self.ctx, first, count, _ptr(pl, i32p), res.ctypes.data, C.byref(js),
                                         C.byref(off)))
        return (pl, res) + self._json_view(js, off, count)

    @staticmethod
    def _json_view(js, off, count):
        offsets = np.ctypeslib.as_array(off, shape=(3 * count + 1,)).copy()
        total = int(offsets[-1])
        buf = (C.c_char * max(total, 1)).from_address(js.value) if total else (C.c_char * 1)()
        return memoryview(buf).cast("B")[:total].toreadonly(), offsets

    def run_queue_json_async(self, first: int, count: int):
        """ksg_run_queue_json_async: placements, results and a ticket; the
        values' copy back is in flight (json_wait(ticket, count))."""
        pl = np.zeros(count, np.int32)
        res = np.zeros(count, RESULT_DTYPE)
        t = C.c_int32()
        self._check(self._run_queue_json_async(self.ctx, first, count, _ptr(pl, i32p), res.ctypes.data,
                                               C.byref(t)))
        return pl, res, t.value

    def json_wait(self, ticket: int, count: int):
        """ksg_json_wait: (values memoryview, offsets) of a launched chunk,
        valid until the third launch after it."""
        js = C.c_void_p()
        off = C.POINTER(C.c_int64)()
        self._check(self._json_wait(self.ctx, ticket, C.byref(js), C.byref(off)))
        return self._json_view(js, off, count)

    def run_replicas(self, profiles, first: int, count: int):
        R = len(profiles)
        arr = (KsgProfile * R)(*[make_profile(p) for p in profiles])
        pl = np.zeros((R, count), np.int32)
        sums = np.zeros(R, SUMMARY_DTYPE)
        self._check(self._run_replicas(self.ctx, arr, R, first, count, _ptr(pl, i32p), sums.ctypes.data))
        return pl, sums

    def set_timing(self, on: bool):
        """Per-kernel HIP-event timing of the following runs (ksg_set_timing)."""
        self._check(self._set_timing(self.ctx, 1 if on else 0))

    def kernel_stats(self):
        """[{name, calls, total_ms, avg_ms, units}] of the last run (timing on)."""
        buf = (KsgKernelStat * 16)()
        n = C.c_int32()
        self._check(self._kernel_stats(self.ctx, buf, 16, C.byref(n)))
        out = []
        for i in range(min(n.value, 16)):
            k = buf[i]
            out.append({"name": k.name.decode(), "calls": k.calls, "total_ms": k.total_ms,
                        "avg_ms": k.total_ms / max(k.calls, 1), "units": k.units})
        return out

    def last_run_info(self):
        """(path, flags) of the last run (ksg_last_run_info): path 1 queue
        kernel, 2 batched, 3 replica sweep, 4 chip-wide topology; flags
        RUN_NARROW_SWEEP / RUN_SLOT32."""
        p, fl = C.c_int32(), C.c_int32()
        self._check(self._run_info(self.ctx, C.byref(p), C.byref(fl)))
        return p.value, fl.value

    def recoveries(self) -> int:
        """Grid-barrier timeouts recovered by a cooperative relaunch (ksg_recoveries)."""
        n = C.c_int32()
        self._check(self._recoveries(self.ctx, C.byref(n)))
        return n.value

    def topo_window_stats(self):
        """(windows, pods decided, windows ended early) of the last run's
        speculative topology queue (ksg_topo_window_stats; zeros on other paths)."""
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        self._check(self._win_stats(self.ctx, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def last_kernel_ms(self) -> float:
        v = C.c_double()
        self._check(self._last_ms(self.ctx, C.byref(v)))
        return v.value

    def read_state(self, n_res: int):
        N = self.n_nodes
        req = np.zeros((n_res, N), np.int64)
        nz = np.zeros((2, N), np.int64)
        pc = np.zeros(N, np.int32)
        st = KsgNodeState(_ptr(req, i64p), _ptr(nz, i64p), _ptr(pc, i32p))
        self._check(self._read_state(self.ctx, C.byref(st)))
        return req, nz, pc

    def reset_state(self):
        self._check(self._reset_state(self.ctx))


# ---- bulk result-store serialiser (host code in libksched.so) ----------------
class KsgNames(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("node", C.POINTER(C.c_char_p)), ("plugin", C.POINTER(C.c_char_p)),
                ("n_res", C.c_int32), ("res", C.POINTER(C.c_char_p)), ("n_taint_vocab", C.c_int32),
                ("taint", C.POINTER(C.c_char_p)), ("max_taints", C.c_int32), ("taints", u32p)]


class KsgAnnotateIn(C.Structure):
    _fields_ = [("n_filter", C.c_int32), ("filter_order", i32p), ("n_score", C.c_int32), ("score_order", i32p),
                ("normalize_mask", C.c_uint32), ("weight", i64p), ("n_feasible", C.c_int32),
                ("fstatus", u32p), ("raw", i64p), ("norm", i64p)]


# a read-only memoryview of `n` bytes at address `p` (PyMemoryView_FromMemory, PyBUF_READ)
_memview = C.pythonapi.PyMemoryView_FromMemory
_memview.restype = C.py_object
_memview.argtypes = [C.c_void_p, C.c_ssize_t, C.c_int]


def _view_at(p, n):
    return _memview(p, n, 0x100) if n else memoryview(b"")


class KsgAnnotateInAt(C.Structure):
    """ksg_annotate_in with its pointers as plain addresses (Annotator.annotate_at)."""
    _fields_ = [("n_filter", C.c_int32), ("filter_order", C.c_void_p), ("n_score", C.c_int32),
                ("score_order", C.c_void_p), ("normalize_mask", C.c_uint32), ("weight", C.c_void_p),
                ("n_feasible", C.c_int32), ("fstatus", C.c_void_p), ("raw", C.c_void_p), ("norm", C.c_void_p)]


def _cstrs(items):
    arr = (C.c_char_p * max(len(items), 1))()
    for i, s in enumerate(items):
        arr[i] = s.encode("utf-8", errors="surrogatepass")
    return arr


class Annotator:
    """ksg_annotator: filter-result / score-result / finalscore-result JSON of
    one pod straight from its capture SoA (resultstore.Store output bytes)."""

    def __init__(self, node_names, plugin_names, res_names, taint_strings, taints: np.ndarray,
                 lib_path: Optional[str] = None):
        path = lib_path or LIB_PATH
        if not os.path.exists(path):
            raise KschedError(f"{path} not found: run __graft_entry__.build()")
        self.lib = C.CDLL(path)
        f = _bind(self.lib, "ksg_")
        self._new = f("annotator_new", C.c_int, C.POINTER(KsgNames), C.POINTER(C.c_void_p))
        self._free = f("annotator_free", C.c_int, C.c_void_p)
        self._annotate = f("annotate", C.c_int, C.c_void_p, C.POINTER(KsgAnnotateIn),
                           C.POINTER(C.c_char_p), C.POINTER(C.c_int64))
        # the same entry point, its strings taken as plain addresses (annotate_views)
        self._annotate_v = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(KsgAnnotateIn), C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_int64))(("ksg_annotate", self.lib))
        self._annotate_at = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_int64))(("ksg_annotate", self.lib))
        self._in_at = KsgAnnotateInAt()
        self._in_at_ref = C.addressof(self._in_at)
        self._out_at = ((C.c_void_p * 3)(), (C.c_int64 * 3)())
        self._keep = [_cstrs(node_names), _cstrs(plugin_names), _cstrs(res_names), _cstrs(taint_strings),
                      np.ascontiguousarray(taints, np.uint32)]
        names = KsgNames(len(node_names), self._keep[0], self._keep[1], len(res_names), self._keep[2],
                         len(taint_strings), self._keep[3], int(self._keep[4].shape[0]),
                         _ptr(self._keep[4], u32p))
        self.h = C.c_void_p()
        rc = self._new(C.byref(names), C.byref(self.h))
        if rc != 0:
            raise KschedError(f"ksg_annotator_new rc={rc}")
        self.n_nodes = len(node_names)
        track(self)

    def annotate(self, filter_order, score_order, normalize_mask: int, weight, n_feasible: int,
                 fstatus: np.ndarray, raw: np.ndarray, norm: np.ndarray):
        return tuple(b.decode("utf-8") for b in self.annotate_bytes(
            filter_order, score_order, normalize_mask, weight, n_feasible, fstatus, raw, norm))

    def annotate_bytes(self, filter_order, score_order, normalize_mask: int, weight, n_feasible: int,
                       fstatus: np.ndarray, raw: np.ndarray, norm: np.ndarray):
        fo = np.ascontiguousarray(filter_order, np.int32)
        so = np.ascontiguousarray(score_order, np.int32)
        w = np.ascontiguousarray(weight, np.int64)
        fs = np.ascontiguousarray(fstatus, np.uint32)
        rw = np.ascontiguousarray(raw, np.int64)
        nm = np.ascontiguousarray(norm, np.int64)
        inp = KsgAnnotateIn(len(fo), _ptr(fo, i32p), len(so), _ptr(so, i32p), normalize_mask, _ptr(w, i64p),
                            n_feasible, _ptr(fs, u32p), _ptr(rw, i64p), _ptr(nm, i64p))
        out = (C.c_char_p * 3)()
        ln = (C.c_int64 * 3)()
        rc = self._annotate(self.h, C.byref(inp), out, ln)
        if rc != 0:
            raise KschedError(f"ksg_annotate rc={rc}")
        return tuple(C.string_at(out[i], ln[i]) for i in range(3))

    def annotate_views(self, filter_order, score_order, normalize_mask: int, weight, n_feasible: int,
                       fstatus: np.ndarray, raw: np.ndarray, norm: np.ndarray):
        """annotate_bytes' values as read-only memoryviews of the annotator's
        own buffers, valid until its next call (as the C strings are): nothing
        is copied, so worker threads serialise in parallel (string_at copied
        every value under the GIL)."""
        fo = np.ascontiguousarray(filter_order, np.int32)
        so = np.ascontiguousarray(score_order, np.int32)
        w = np.ascontiguousarray(weight, np.int64)
        fs = np.ascontiguousarray(fstatus, np.uint32)
        rw = np.ascontiguousarray(raw, np.int64)
        nm = np.ascontiguousarray(norm, np.int64)
        inp = KsgAnnotateIn(len(fo), _ptr(fo, i32p), len(so), _ptr(so, i32p), normalize_mask, _ptr(w, i64p),
                            n_feasible, _ptr(fs, u32p), _ptr(rw, i64p), _ptr(nm, i64p))
        out = (C.c_void_p * 3)()
        ln = (C.c_int64 * 3)()
        rc = self._annotate_v(self.h, C.byref(inp), out, ln)
        if rc != 0:
            raise KschedError(f"ksg_annotate rc={rc}")
        return self._views(out, ln)

    def annotate_at(self, n_filter: int, filter_order: int, n_score: int, score_order: int, normalize_mask: int,
                    weight: int, n_feasible: int, fstatus: int, raw: int, norm: int):
        """annotate_views with every array given as an address the caller keeps
        valid (the bulk path's per-pod call: no conversions, one reused
        argument struct)."""
        a = self._in_at
        a.n_filter, a.filter_order, a.n_score, a.score_order = n_filter, filter_order, n_score, score_order
        a.normalize_mask, a.weight, a.n_feasible = normalize_mask, weight, n_feasible
        a.fstatus, a.raw, a.norm = fstatus, raw, norm
        out, ln = self._out_at
        rc = self._annotate_at(self.h, self._in_at_ref, out, ln)
        if rc != 0:
            raise KschedError(f"ksg_annotate rc={rc}")
        return self._views(out, ln)

    def _views(self, out, ln):
        # read-only views straight onto the annotator's buffers: no copy at all
        return tuple(_view_at(out[i], ln[i]) for i in range(3))

    def close(self):
        if self.h:
            self._free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
