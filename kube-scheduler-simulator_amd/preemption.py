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
PreFilter state instead).  The node-static filters (NodeUnschedulable,
NodeName, TaintToleration, NodeAffinity and the volume plugins) are not
re-run: no removal changes them.  When one of them is ordered after a
pod-dependent filter (VolumeBinding / VolumeZone after NodeResourcesFit in
the default order, for a preemptor with claims), a node whose recorded
rejection is the pod-dependent one may still fail it; the candidate lists
then keep only the nodes `ksg_eval_skipping` passes with the pod-dependent
filters skipped (`static_skip_mask`).  VolumeRestrictions is node-static
except for a ReadWriteOncePod conflict, which removing the claim's holders
clears (its RemovePod extension): `rwop_outcome` decides the cases where no
node can clear it and refuses the one the dry run does not model (every
holder of lower priority on a single node).  Scope (refused with
NotImplementedError, never computed wrongly): that case.  There are no
PodDisruptionBudgets in a snapshot, so every victim is non-violating.
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
    if pl == P.VOLUME_RESTRICTIONS:            # satisfyReadWriteOncePod: Unschedulable
        return UNSCHEDULABLE
    return UNSCHEDULABLE_AND_UNRESOLVABLE      # node-static filters, VolumeBinding, VolumeZone


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


def static_skip_mask() -> int:
    """ksg_eval_skipping's filter_skip for the node-static verdict: the four
    filters the dry run re-runs skipped, so a node's status word is 0 iff
    every other Filter plugin passes it."""
    return sum(1 << p for p in _POD_DEPENDENT)


def needs_static_verdict(prof: P.Profile, pod: m.Pod) -> bool:
    """Whether a potential node (its recorded rejection pod-dependent) can
    still fail a node-static filter ordered after that rejection: some
    static filter follows a pod-dependent one in the profile's order.  The
    volume plugins count only for a preemptor with claims (Skip or pass
    without them)."""
    order = prof.filter_order()
    first = min((order.index(p) for p in _POD_DEPENDENT if p in order), default=None)
    if first is None:
        return False
    late = [p for p in order[first + 1:] if p not in _POD_DEPENDENT]
    if not pod.claim_names():
        late = [p for p in late if p not in E.VOLUME_PLUGINS]
    return bool(late)


def rwop_holders(pod: m.Pod, placed: Sequence[Tuple[int, int, m.Pod]]) -> List[Tuple[int, int]]:
    """(pod index, node) of the placed pods holding one of `pod`'s
    ReadWriteOncePod claims: VolumeRestrictions' conflictingPVCRefCount
    (upstream volumerestrictions PreFilter, StorageInfos.IsPVCUsedByPods).
    `placed` = (index, node, pod) of every placed pod."""
    if pod.storage is None:
        return []
    rwop = set()
    for c in pod.claim_names():
        pvc = pod.storage.claim(pod.namespace, c)
        if pvc is not None and m.READ_WRITE_ONCE_POD in pvc.access_modes:
            rwop.add(c)
    if not rwop:
        return []
    return [(q, n) for q, n, o in placed
            if o is not pod and o.namespace == pod.namespace and rwop & set(o.claim_names())]


def rwop_outcome(pod: m.Pod, holders: Sequence[Tuple[int, int]], pods: Sequence[m.Pod]) -> Optional[int]:
    """A preemptor with a ReadWriteOncePod conflict: removing victims from one
    node clears the conflict (VolumeRestrictions RemovePod) only when every
    holder runs on that node and is a potential victim (lower priority).
    Otherwise VolumeRestrictions rejects the preemptor on every node of the
    dry run and there is no candidate: returns -1.  The remaining case is
    refused: the dry run would have to keep the holders evicted through the
    reprieve."""
    if not holders:
        return None
    if len({n for _, n in holders}) > 1 or any(pods[q].priority >= pod.priority for q, _ in holders):
        return -1
    raise NotImplementedError("DefaultPreemption for a preemptor whose ReadWriteOncePod claim a lower-priority "
                              "pod holds (VolumeRestrictions RemovePod)")


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
