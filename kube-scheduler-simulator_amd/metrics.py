"""Algorithmic byte counts for the roofline.

Bytes per node-eval = every SoA column the enabled plugins must read for one
node, each counted once, plus the per-node bytes written (none in
placement-only mode).  The pod spec (staged once per pod in LDS) and LDS
table lookups are not counted.  `achieved` = bytes/node-eval x node-evals per
launch / launch time.
"""
from __future__ import annotations

from typing import Dict

from . import encoder as E
from . import profile as P

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E vendor peak (MI355X_MICROARCH.md, chip table)


def bytes_per_node_eval(enc: E.Encoder, prof: P.Profile) -> Dict[str, int]:
    en = set(prof.enabled_ids())
    R = len(enc.cluster.res_names)
    cols: Dict[str, int] = {}
    if P.NODE_UNSCHEDULABLE in en:
        cols["unschedulable"] = 1
    if P.NODE_RESOURCES_FIT in en or P.BALANCED_ALLOCATION in en:
        cols["alloc"] = 8 * R
        cols["requested"] = 8 * R
        cols["allowed_pods"] = 4
        cols["pod_count"] = 4
    if P.NODE_RESOURCES_FIT in en:
        cols["nonzero"] = 16
    if P.TAINT_TOLERATION in en:
        cols["taints"] = 4 * enc.cluster.max_taints
    if P.NODE_AFFINITY in en:
        # label columns referenced by node-affinity programs (all label columns
        # that are not pure topology keys)
        na_keys = set()
        for p in enc.pods:
            if p.node_selector:
                na_keys.update(p.node_selector)
            for t in (p.node_affinity_required or []):
                na_keys.update(r.key for r in t.match_expressions)
            for pt in (p.node_affinity_preferred or []):
                na_keys.update(r.key for r in pt.preference.match_expressions)
        cols["labels"] = 4 * len(na_keys)
    if P.IMAGE_LOCALITY in en:
        cols["images"] = 4 * enc.cluster.max_images
    if P.POD_TOPOLOGY_SPREAD in en or P.INTER_POD_AFFINITY in en:
        topo = set()
        for p in enc.pods:
            for c in p.topology_spread_constraints:
                topo.add(c.topology_key)
            for t in p.pod_affinity_required + p.pod_anti_affinity_required:
                topo.add(t.topology_key)
            for w in p.pod_affinity_preferred + p.pod_anti_affinity_preferred:
                topo.add(w.term.topology_key)
        cols["topology_labels"] = 4 * len(topo)
        cols["selector_counts"] = 4     # one per-node count lookup per constraint/term
    return cols


def roofline(bytes_per_eval: int, node_evals_per_launch: int, launch_ms: float) -> Dict[str, float]:
    achieved = bytes_per_eval * node_evals_per_launch / (launch_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS}


# Algorithmic bytes per unit of each kernel (units as ksg_kernel_stats counts them).
#   queue kernels, batch phase 1: one node-eval per (pod, node) = the column
#     schema above; phase 1 also writes its 8-byte record + 4-byte image part
#   topk / scan phase 2: one 8-byte record read per (pod, node)
#   top-set phase 2 (all variants): per unit one 8-byte top key + 8-byte record + 4-byte image part
#   replica sweep, static records (unit = (pod, node)): the replica-independent
#     columns (unschedulable, taints, labels, images) + the 8-byte record written
#   replica sweep (unit = (replica, pod, node)): the 8-byte static record + the
#     Fit / BalancedAllocation columns it reads: allocatable and requested of
#     cpu and memory, non-zero requested, pod count, allowed pods
#   narrow replica sweep: the 8-byte static record + the 16-byte per-node
#     static record + the 16-byte per-(replica, node) record
STATIC_COLS = ("unschedulable", "taints", "labels", "images")


def kernel_bytes_per_unit(name: str, cols) -> int:
    bytes_per_eval = sum(cols.values()) if isinstance(cols, dict) else int(cols)
    if name in ("ksg_queue_kernel", "ksg_queue_topo_kernel", "ksg_topo_coop"):
        return bytes_per_eval
    if name == "ksg_topo_coop_window":   # a window row's node-eval + its 4-byte static total written
        return bytes_per_eval + 4      # (the walk's reads are O(window), not O(nodes))
    if name == "ksg_batch_phase1":
        return bytes_per_eval + 12
    if name == "ksg_capture_eval":   # node columns on the post-batch state + status word and record written
        return bytes_per_eval + 12
    if name == "ksg_capture_norm":   # record read, normalised row and total written (one scored row at least)
        return 24
    if name == "ksg_eval_cycle":     # ksg_capture_eval + ksg_capture_norm in one launch (per-cycle path)
        return bytes_per_eval + 12 + 24
    if name == "ksg_batch_topk":
        return 8
    if name in ("ksg_batch_phase2s", "ksg_batch_phase2v"):
        return 20
    if name in ("ksg_sweep_static", "ksg_sweep"):
        if not isinstance(cols, dict):
            raise TypeError("the replica-sweep kernels need the per-column byte counts")
        if name == "ksg_sweep_static":
            return sum(cols.get(k, 0) for k in STATIC_COLS) + 8
        fit = 32 if "alloc" in cols else 0
        return 8 + fit + sum(cols.get(k, 0) for k in ("nonzero", "pod_count", "allowed_pods"))
    if name == "ksg_sweep_narrow":
        return 40
    raise KeyError(name)


def dominant_kernel_roofline(kstats, bytes_per_eval):
    """Roofline of the kernel with the largest summed time: algorithmic bytes
    per launch / average launch duration; every kernel listed under "kernels"."""
    if not kstats:
        return None
    rows = []
    for k in kstats:
        bpu = kernel_bytes_per_unit(k["name"], bytes_per_eval)
        per_launch = bpu * k["units"] / max(k["calls"], 1)
        r = roofline(1, per_launch, k["avg_ms"]) if k["avg_ms"] > 0 else {"achieved": 0.0, "frac": 0.0}
        rows.append({"name": k["name"], "calls": k["calls"], "avg_ms": k["avg_ms"], "total_ms": k["total_ms"],
                     "bytes_per_launch": per_launch, "bytes_per_unit": bpu,
                     "achieved": r["achieved"], "frac": r["frac"]})
    dom = max(rows, key=lambda r: r["total_ms"])
    return {"bound": "hbm", "achieved": dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": dom["frac"], "kernel": dom["name"], "avg_launch_ms": dom["avg_ms"],
            "bytes_per_launch": dom["bytes_per_launch"], "kernels": rows}


PHASE2_KERNELS = ("ksg_batch_phase2s", "ksg_batch_phase2v")


def price_decided_node_evals(roof, bytes_per_eval: int, node_evals: int):
    """A phase-2 walk decides a batch of pods over every node: price a launch
    by SURVEY §8(d)'s bytes per node-eval x the node-evals it decides (batch
    pods x nodes, i.e. node_evals of the run / launches), as the round-1
    verdict recomputed it; the changed-slot figure the kernel stats count is
    kept as achieved_changed_slot_bytes."""
    if not roof or roof.get("kernel") not in PHASE2_KERNELS:
        return roof
    row = next((k for k in roof.get("kernels", []) if k["name"] == roof["kernel"]), None)
    if row and row["calls"] and row["avg_ms"] > 0:
        per_launch = bytes_per_eval * node_evals / row["calls"]
        roof["achieved_changed_slot_bytes"] = roof["achieved"]
        roof["achieved"] = per_launch / (row["avg_ms"] * 1e-3) / 1e9
        roof["frac"] = roof["achieved"] / roof["peak"]
        roof["bytes_per_launch"] = per_launch
        roof["unit_basis"] = "SURVEY 8(d) bytes per node-eval x node-evals decided per launch (batch pods x nodes)"
    return roof
