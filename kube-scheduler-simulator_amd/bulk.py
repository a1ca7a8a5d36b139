"""Bulk annotation: a whole queue's filter-result / score-result /
finalscore-result values (store.go:423-507 as GetStoredResult serialises them,
store.go:133-198) from one captured device run.

`framework.DebuggableScheduler` mirrors the wrapper pod by pod (one ksg_eval,
record, commit per cycle).  For a queue that needs no preemption the same
three annotation values come out of one captured `ksg_run_queue` (the batched
path with its capture kernels, ksched_capture.h) followed by one
`ksg_annotate` per pod; `annotate_queue` runs that in chunks, with the device
capture of chunk i + 1 overlapping the native serialisation of chunk i on a
thread pool (ctypes releases the GIL in both calls).  The bytes are the
per-pod path's, which tests/test_gpu_bulk_annotations.py checks.
"""
from __future__ import annotations

import itertools
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional

import numpy as np

from . import encoder as E
from . import native
from . import profile as P


class BulkAnnotator:
    """Per-profile constants plus one native annotator per worker thread."""

    def __init__(self, enc: E.Encoder, prof: P.Profile, threads: int = 1):
        cl = enc.cluster
        self.enc, self.prof = enc, prof
        self.n_nodes = len(cl.node_names)
        taints = [f"{{{t.key}: {t.value}}}" for t in cl.taint_vocab]
        self.annotators = [native.Annotator(cl.node_names, P.PLUGIN_NAMES, cl.res_names, taints, cl.arrays["taints"])
                           for _ in range(max(1, threads))]
        store_w = prof.weights()
        self.weights = np.array([store_w.get(n, 0) for n in P.PLUGIN_NAMES], np.int64)
        self._w_addr = self.weights.ctypes.data
        self.norm_mask = sum(1 << pid for pid in range(len(P.PLUGIN_NAMES)) if P.EXT[pid][4])
        self.filter_order = prof.filter_order()
        self.score_order = prof.score_order()
        self.fskip = enc.workload.pods["filter_skip"].astype(np.int64).tolist()
        self._orders = {}   # (filter skips, score skips or -1) -> (arrays, lengths, addresses)
        self.pool = ThreadPoolExecutor(max_workers=len(self.annotators)) if len(self.annotators) > 1 else None

    def close(self):
        if self.pool:
            self.pool.shutdown()
        for a in self.annotators:
            a.close()

    def _order(self, fskip: int, sskip: int):
        """The plugins that ran, per (filter skips, score skips), as int32 arrays
        kept alive here with their addresses (a few distinct keys per queue)."""
        key = (fskip, sskip)
        v = self._orders.get(key)
        if v is None:
            fo = np.array([p for p in self.filter_order if not (fskip >> p) & 1], np.int32)
            so = np.array([p for p in self.score_order if not (sskip >> p) & 1] if sskip >= 0 else [], np.int32)
            v = (fo, so, len(fo), fo.ctypes.data, len(so), so.ctypes.data)
            self._orders[key] = v
        return v

    def _pod(self, ann: native.Annotator, k: int, pi: int, res, cap: native.CaptureBuffers):
        st, nf, sskip = int(res["status"][k]), int(res["n_feasible"][k]), int(res["score_skip"][k])
        return self._pod_at(ann, k, pi, st, nf, sskip, cap)

    def _pod_at(self, ann: native.Annotator, k: int, pi: int, status: int, nf: int, sskip: int,
                cap: native.CaptureBuffers):
        fskip = self.fskip[pi]
        if status & native.ST_IPA_PREFILTER_SKIP:
            fskip |= 1 << P.INTER_POD_AFFINITY
        _, _, nfo, fo, nso, so = self._order(fskip, sskip if nf >= 2 else -1)
        N = self.n_nodes
        return ann.annotate_at(nfo, fo, nso, so, self.norm_mask, self._w_addr, nf,
                               cap.fstatus.ctypes.data + 4 * N * k, cap.raw.ctypes.data + 8 * native.NPLUGINS * N * k,
                               cap.norm.ctypes.data + 8 * native.NPLUGINS * N * k)

    def serialise(self, first: int, res, cap: native.CaptureBuffers, count: int,
                  sink: Callable[[int, tuple], None]):
        """ksg_annotate for pods first .. first + count of a captured chunk;
        sink(pod index, (filter, score, finalscore)), increasing per worker; the
        values are read-only memoryviews valid for the sink call only (bytes(v)
        keeps one; hash.update(v) reads it in place)."""
        T = len(self.annotators)
        status, nfeas, sskip = (res[f][:count].tolist() for f in ("status", "n_feasible", "score_skip"))
        assert cap.fstatus.shape == (cap.fstatus.shape[0], self.n_nodes) and count <= cap.fstatus.shape[0]

        nxt = itertools.count()   # pods handed out one at a time (their sizes differ)

        def work(t):
            ann = self.annotators[t]
            for k in iter(nxt.__next__, None):
                if k >= count:
                    return
                sink(first + k, self._pod_at(ann, k, first + k, status[k], nfeas[k], sskip[k], cap))

        if self.pool is None:
            work(0)
        else:
            list(self.pool.map(work, range(T)))


def annotate_queue(engine: native.Engine, bulk: BulkAnnotator, first: int, count: int,
                   sink: Callable[[int, tuple], None], chunk: int = 256) -> np.ndarray:
    """Schedule pods [first, first + count) in chunks with capture on, emitting
    every pod's three annotation values through `sink`; returns placements.
    The device capture of the next chunk overlaps the serialisation of the
    current one."""
    N = bulk.n_nodes
    out = np.empty(count, np.int32)
    io = ThreadPoolExecutor(max_workers=1)
    caps = [native.CaptureBuffers(N, min(chunk, count)) for _ in range(2)]

    def capture(off, buf):
        k = min(chunk, count - off)
        pl, res = engine.run_queue(first + off, k, capture=buf)
        return off, k, pl, res, buf

    pending: Optional[object] = io.submit(capture, 0, caps[0]) if count else None
    i = 0
    while pending is not None:
        off, k, pl, res, buf = pending.result()
        out[off:off + k] = pl
        nxt = off + k
        i ^= 1
        pending = io.submit(capture, nxt, caps[i]) if nxt < count else None
        bulk.serialise(first + off, res, buf, k, sink)
    io.shutdown()
    return out


def annotate_queue_device(engine: native.Engine, bulk: BulkAnnotator, first: int, count: int,
                          sink: Callable[[int, tuple], None], chunk: int = 256) -> np.ndarray:
    """annotate_queue with the values serialised on the device
    (ksg_run_queue_json_async, csrc/ksched_json.h): per chunk one captured
    run whose capture rows never leave HBM, the finished bytes copied back on
    a stream of their own.  Chunk i's sink (on the annotator's worker
    threads) overlaps chunk i + 1's copy back and chunk i + 2's run (three
    pinned buffers rotate in the library).  Pods the capture paths do not take
    (host ports, claims) are refused by the library: use annotate_queue."""
    engine.attach_annotator(bulk.annotators[0], bulk.weights, bulk.norm_mask)
    out = np.empty(count, np.int32)
    offs_of = list(range(0, count, chunk))
    io = ThreadPoolExecutor(max_workers=1)

    def launch(j):
        off = offs_of[j]
        k = min(chunk, count - off)
        pl, _, t = engine.run_queue_json_async(first + off, k)
        out[off:off + k] = pl
        return off, k, t

    try:
        launched = [launch(j) for j in range(min(2, len(offs_of)))]
        for j in range(len(offs_of)):
            off, k, t = launched[j]
            js, offs = engine.json_wait(t, k)
            fut = io.submit(launch, j + 2) if j + 2 < len(offs_of) else None

            def emit(i, js=js, offs=offs, base=first + off):
                o = offs[3 * i: 3 * i + 4]
                sink(base + i, (js[o[0]:o[1]], js[o[1]:o[2]], js[o[2]:o[3]]))

            if bulk.pool is None:
                for i in range(k):
                    emit(i)
            else:
                list(bulk.pool.map(emit, range(k)))
            if fut is not None:
                launched.append(fut.result())
    finally:
        io.shutdown()
    return out
