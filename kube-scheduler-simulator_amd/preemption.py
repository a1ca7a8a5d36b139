"""DefaultPreemption PostFilter: the host half of the device dry run.

The simulator wraps the upstream plugin (`wrappedplugin.go:550-583`) and
records the nominated node into the store (`store.go:442-458`).  The plugin
itself is upstream v1.32 (`pkg/scheduler/framework/plugins/defaultpreemption`
and `framework/preemption`, `k8s.io/kubernetes v1.32.5`, not vendored).  Its
steps, and where each one runs here:

1. `PodEligibleToPreemptOthers`: `preemptionPolicy: Never` pods do not
   preempt (host; no pod is ever left nominated in this model, see 6).
2. `findCandidates`: potential nodes are the nodes whose filter status is
   `Unschedulable` (not `UnschedulableAndUnresolvable`), read from the
   device's filter status words (`status_code`).
3. `DryRunPreemption` / `SelectVictimsOnNode`: for every potential node,
   remove the pods of lower priority, re-run the filters, reprieve the
   victims most important first.  That is `ksg_preempt_victims`, one lane per
   node on the GPU.  Upstream visits the potential nodes from a random offset
   in parallel and stops after `num_candidates` candidates; here the visit
   starts at offset 0 and candidates are taken in node order (the seeded
   deterministic choice, like selectHost's lowest-index tie-break).
4. `SelectCandidate` / `pickOneNodeForPreemption`: fewest PDB violations,
   lowest highest victim priority, lowest priority sum, fewest victims,
   latest earliest start time; a remaining tie (Go map order upstream) goes
   to the lowest node index (`pick_one_node`).
5. `prepareCandidate`: the victims are deleted (`ksg_uncommit`).
6. The preemptor is nominated.  The model retries it at once: the victims'
   deletion events move it back to the active queue, where PrioritySort puts
   it ahead of every pod of lower or equal priority still queued.  The retry
   evaluates the nominated node first (`schedule_one.go`
   `evaluateNominatedNode`): when it passes, it is the only feasible node and
   the pod binds there without scoring.

The dry run re-runs the filters that read the node's pods: NodeResourcesFit,
NodePorts (a preemptor with host ports: the node's UsedPorts as the removed /
reprieved victims leave them, set semantics as upstream's HostPortInfo) and,
for a preemptor with hard spread constraints or required inter-pod terms
(or matched by existing pods' anti-affinity), PodTopologySpread and
InterPodAffinity with the PreFilter counts of the candidate's domains moved by
the removed / reprieved pods (ksched_preempt.h; the oracles recompute the
PreFilter state instead).  Scope (refused with NotImplementedError, never
computed wrongly): profiles that order a node-static filter after one of those
three.  There are no PodDisruptionBudgets in a snapshot, so every victim is
non-violating.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from . import encoder as E
from . import model as m
from . import profile as P

SUCCESS, ERROR, UNSCHEDULABLE, UNSCHEDULABLE_AND_UNRESOLVABLE = 0, 1, 2, 3

# util.GetPodStartTime answers time.Now() for a pod without status.startTime:
# later than every recorded start, equal among such pods.
NOW = 1 << 62
INT32_SPAN = 1 << 31          # math.MaxInt32 + 1 (minSumPrioritiesScoreFunc)

_STATIC_FILTERS = (P.NODE_UNSCHEDULABLE, P.NODE_NAME, P.TAINT_TOLERATION, P.NODE_AFFINITY)


def status_code(word: int, req=None, alloc=None) -> int:
    """framework.Code of a node's filter result from its device status word
    (plugin id + 1 in bits 0-7, reason above).  Nodes outside the PreFilter
    node set (FS_NOT_EVALUATED) carry the absent-nodes status.  For
    NodeResourcesFit, `req` (the pod's request per resource column) and
    `alloc` (the node's allocatable) give InsufficientResource.Unresolvable:
    a request above the allocatable outright (framework.status_code)."""
    if word == 0:
        return SUCCESS
    if word == E.FS_NOT_EVALUATED:
        return UNSCHEDULABLE_AND_UNRESOLVABLE
    pl, reason = (word & 0xFF) - 1, word >> 8
    if pl == P.NODE_RESOURCES_FIT:
        if req is not None:
            for r in range(len(alloc)):
                if reason & (1 << (r + 1)) and int(req[r]) > int(alloc[r]):
                    return UNSCHEDULABLE_AND_UNRESOLVABLE
        return UNSCHEDULABLE
    if pl == P.NODE_PORTS:
        return UNSCHEDULABLE
    if pl == P.POD_TOPOLOGY_SPREAD:            # ErrReasonNodeLabelNotMatch is unresolvable
        return UNSCHEDULABLE_AND_UNRESOLVABLE if reason == 1 else UNSCHEDULABLE
    if pl == P.INTER_POD_AFFINITY:             # ErrReasonAffinityRulesNotMatch is unresolvable
        return UNSCHEDULABLE_AND_UNRESOLVABLE if reason == 1 else UNSCHEDULABLE
    return UNSCHEDULABLE_AND_UNRESOLVABLE      # NodeUnschedulable, NodeName, TaintToleration, NodeAffinity


def start_of(pod: m.Pod) -> int:
    return pod.start_time if pod.start_time is not None else NOW


def importance_key(pod: m.Pod):
    """Ascending order = util.MoreImportantPod (higher priority, then earlier
    start).  Upstream sorts with the unstable sort.Slice; equal pods are
    ordered by namespace/name here."""
    return (-pod.priority, start_of(pod), pod.namespace, pod.name)


def num_candidates(n_potential: int, prof: P.Profile) -> int:
    """DefaultPreemption.calculateNumCandidates."""
    n = n_potential * prof.preemption_min_candidate_pct // 100
    n = max(n, prof.preemption_min_candidate_abs)
    return min(n, n_potential)


def earliest_start_of_highest(victims: Sequence[m.Pod]) -> Optional[int]:
    """util.GetEarliestPodStartTime."""
    if not victims:
        return None
    best, top = start_of(victims[0]), victims[0].priority
    for v in victims:
        if v.priority == top:
            best = min(best, start_of(v))
        elif v.priority > top:
            top, best = v.priority, start_of(v)
    return best


def pick_one_node(cands: Sequence[Tuple[int, Sequence[m.Pod], int]]) -> int:
    """pickOneNodeForPreemption over (node, victims most important first,
    PDB violations); returns the node."""
    funcs = (
        lambda c: -c[2],
        lambda c: -c[1][0].priority,
        lambda c: -sum(v.priority + INT32_SPAN for v in c[1]),
        lambda c: -len(c[1]),
        lambda c: earliest_start_of_highest(c[1]),
    )
    pool = sorted(cands, key=lambda c: c[0])
    for f in funcs:
        best = max(f(c) for c in pool)
        pool = [c for c in pool if f(c) == best]
        if len(pool) == 1:
            break
    return pool[0][0]


_POD_DEPENDENT = (P.NODE_RESOURCES_FIT, P.NODE_PORTS, P.POD_TOPOLOGY_SPREAD, P.INTER_POD_AFFINITY)


def check_scope(prof: P.Profile, pod: m.Pod, pods: Sequence[m.Pod]) -> None:
    """Refuse preemption the dry run cannot decide exactly: it re-runs the
    filters that read the node's pods (Fit, NodePorts, PodTopologySpread,
    InterPodAffinity), so every node-static filter must come before them."""
    if pod.claim_names() and set(prof.filter_order()) & {P.VOLUME_RESTRICTIONS, P.VOLUME_BINDING, P.VOLUME_ZONE}:
        # the dry run re-runs Fit / PTS / IPA only; VolumeRestrictions' AddPod /
        # RemovePod extensions (ReadWriteOncePod users) are not modelled
        raise NotImplementedError("DefaultPreemption for a preemptor with claims (volume plugins)")
    order = prof.filter_order()
    first = min((order.index(p) for p in _POD_DEPENDENT if p in order), default=None)
    if first is not None:
        late = [P.PLUGIN_NAMES[p] for p in order[first + 1:] if p in _STATIC_FILTERS]
        if late:
            raise NotImplementedError(f"DefaultPreemption with {late} ordered after {P.PLUGIN_NAMES[order[first]]}")


def potential_nodes(fstatus, req=None, alloc=None) -> List[int]:
    """nodesWherePreemptionMightHelp; req = the pod's request columns, alloc
    = [n_res][n_nodes] allocatable."""
    return [n for n in range(len(fstatus))
            if status_code(int(fstatus[n]), req, None if alloc is None else alloc[:, n]) == UNSCHEDULABLE]


def may_preempt(pod: m.Pod, placed_min_priority: Optional[int]) -> bool:
    """Whether `pod` could find a victim among pods whose lowest priority is
    `placed_min_priority` (None: no pod placed)."""
    return (pod.preemption_policy != "Never" and placed_min_priority is not None
            and pod.priority > placed_min_priority)
