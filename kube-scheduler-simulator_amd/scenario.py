"""Scenario-based simulation (KEP-140) and SchedulerSimulation what-ifs
(KEP-184) over the device evaluator: SURVEY §8(f) row 4, the scheduling
queue's requeue semantics plus a scenario driver.

The reference specifies both in its KEPs, not in code:
keps/140-scenario-based-simulation/README.md (the Scenario CRD :62-326, the
ScenarioStep concept :402-523) and keps/184-scheduler-simulation/README.md
(one Scenario, run under several schedulers).  Here:

* `load_scenario(doc)` reads a Scenario's `spec.operations`
  (createOperation / deleteOperation / doneOperation with their MajorStep
  `step`; patchOperation is refused) from a dict or JSON text.
* `ScenarioRunner.run(ops)` plays them step by step.  At MajorStep X the
  operations of X run in order, then the scheduler (the SimulationController)
  runs until nothing it can do changes the cluster, and the step ends.  Every
  resource operation, the scheduler's included, advances the MinorStep.
* The queue is the upstream PriorityQueue with its clock removed.  activeQ is
  a heap in PrioritySort order (priority, then the order pods entered the
  queue).  A pod that fails moves to the unschedulable set together with the
  plugins that rejected it (diagnosis.UnschedulablePlugins: each node's first
  rejecting plugin, from the device status words).  A cluster event (node
  added or deleted, assigned pod added or deleted) moves back to activeQ
  exactly the pods rejected by a plugin registered for that event
  (`REGISTERED`, the plugins' EventsToRegister at event granularity; the
  QueueingHint functions' finer per-object checks are not modelled).  Backoff
  and the periodic flush of unschedulable pods are timers, with no
  counterpart in a step-driven simulation.
* Each attempt's result set is reflected onto the pod as the storereflector
  does (`result-history` keeps every attempt, across steps).
* `ScenarioResult.timeline` holds the operations plus the scheduler's own
  `podScheduled` and preemption `delete` events, keyed by MajorStep.
* `simulate(doc, profiles, make_engine, rank, world)` runs one scenario under
  several scheduler profiles: contiguous blocks of profiles per rank (one
  process per GPU), one all_gather_object of the results at the end.

The cluster changes between steps (operations), so each step encodes the
current cluster once and loads it into a fresh engine; within a step every
cycle is one device evaluation (plus DefaultPreemption's dry run).
"""
from __future__ import annotations

import heapq
import json
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

from . import framework as F
from . import ingest as I
from . import model as m
from . import profile as P

NODE_ADD, NODE_DELETE, POD_ADD, POD_DELETE = "NodeAdd", "NodeDelete", "AssignedPodAdd", "AssignedPodDelete"

# Cluster events each Filter plugin registers for (upstream v1.32
# EventsToRegister, restricted to the events a scenario produces).
REGISTERED = {
    P.NODE_UNSCHEDULABLE: {NODE_ADD},
    P.NODE_NAME: {NODE_ADD},
    P.TAINT_TOLERATION: {NODE_ADD},
    P.NODE_AFFINITY: {NODE_ADD},
    P.NODE_PORTS: {NODE_ADD, POD_DELETE},
    P.NODE_RESOURCES_FIT: {NODE_ADD, POD_DELETE},
    P.POD_TOPOLOGY_SPREAD: {NODE_ADD, NODE_DELETE, POD_ADD, POD_DELETE},
    P.INTER_POD_AFFINITY: {NODE_ADD, POD_ADD, POD_DELETE},
}


@dataclass
class Operation:
    """One ScenarioOperation (KEP-140 :121-177)."""
    id: str
    step: int
    create: Optional[dict] = None          # the object to create (Node or Pod JSON)
    delete: Optional[tuple] = None         # (kind, namespace, name)
    done: bool = False


def load_scenario(doc) -> List[Operation]:
    if isinstance(doc, (str, bytes)):
        doc = json.loads(doc)
    spec = doc.get("spec", doc)
    ops = []
    for k, o in enumerate(spec.get("operations") or ()):
        op = Operation(id=o.get("id") or f"op-{k}", step=int(o.get("step", 0)))
        kinds = [x for x in ("createOperation", "patchOperation", "deleteOperation", "doneOperation") if o.get(x)
                 is not None]
        if len(kinds) != 1:
            raise ValueError(f"operation {op.id}: exactly one of create/patch/delete/done must be set")
        if kinds[0] == "patchOperation":
            raise NotImplementedError("patchOperation")
        if kinds[0] == "createOperation":
            op.create = o["createOperation"]["object"]
            if op.create.get("kind") not in ("Node", "Pod"):
                raise NotImplementedError(f"createOperation of kind {op.create.get('kind')!r}")
        elif kinds[0] == "deleteOperation":
            d = o["deleteOperation"]
            kind = (d.get("typeMeta") or {}).get("kind")
            if kind not in ("Node", "Pod"):
                raise NotImplementedError(f"deleteOperation of kind {kind!r}")
            meta = d.get("objectMeta") or {}
            op.delete = (kind, meta.get("namespace") or "default", meta["name"])
        else:
            op.done = True
        ops.append(op)
    return sorted(ops, key=lambda o: o.step)    # stable: spec order within a step


@dataclass
class _PodState:
    pod: m.Pod
    ordinal: int                     # order of entering the queue (PrioritySort tie-break)
    node: str = ""                   # bound node, "" pending
    rejectors: Optional[set] = None  # None: in activeQ; else the plugins that rejected it
    attempts: int = 0
    annotations: Dict[str, str] = field(default_factory=dict)


class ScenarioRunner:
    """Runs one scenario under one scheduler profile."""

    def __init__(self, prof: P.Profile, make_engine: Callable[[], object], native_annotations: bool = True):
        self.prof = prof
        self.make_engine = make_engine
        self.native_annotations = native_annotations
        self.nodes: List[m.Node] = []
        self.pods: Dict[str, _PodState] = {}
        self.timeline: Dict[str, List[dict]] = {}
        self.major = 0
        self.minor = 0
        self._ordinal = 0
        self._nsched = 0
        self._npre = 0

    # ---- timeline -------------------------------------------------------
    def _event(self, ev: dict) -> None:
        ev["step"] = {"major": self.major, "minor": self.minor}
        self.timeline.setdefault(str(self.major), []).append(ev)
        self.minor += 1

    def _wake(self, event: str) -> None:
        """Move the unschedulable pods a plugin of theirs registered `event` for back to activeQ."""
        for ps in self.pods.values():
            if not ps.node and ps.rejectors is not None and any(event in REGISTERED.get(p, ()) for p in ps.rejectors):
                ps.rejectors = None

    # ---- operations -----------------------------------------------------
    def _apply(self, op: Operation) -> None:
        if op.done:
            self._event({"id": op.id, "done": {"operation": {}}})
            return
        if op.create is not None:
            obj = op.create
            if obj["kind"] == "Node":
                node = I.node_from_k8s(obj)
                if any(n.name == node.name for n in self.nodes):
                    raise ValueError(f"node {node.name} exists")
                self.nodes.append(node)
                self._event({"id": op.id, "create": {"operation": {"object": obj}}})
                self._wake(NODE_ADD)
            else:
                pod = I.pod_from_k8s(obj)
                pod.priority = int((obj.get("spec") or {}).get("priority") or 0)
                pod.preemption_policy = (obj.get("spec") or {}).get("preemptionPolicy") or "PreemptLowerPriority"
                pod.start_time = I.rfc3339_ns((obj.get("status") or {}).get("startTime"))
                key = f"{pod.namespace}/{pod.name}"
                if key in self.pods:
                    raise ValueError(f"pod {key} exists")
                ps = _PodState(pod, self._ordinal)
                self._ordinal += 1
                if pod.node_name:     # bypasses the scheduler: bound as created
                    if not any(n.name == pod.node_name for n in self.nodes):
                        raise NotImplementedError(f"pod {key} bound to a node that does not exist")
                    ps.node = pod.node_name
                self.pods[key] = ps
                self._event({"id": op.id, "create": {"operation": {"object": obj}}})
                if ps.node:
                    self._wake(POD_ADD)
            return
        kind, ns, name = op.delete
        meta = {"typeMeta": {"kind": kind}, "objectMeta": {"name": name} if kind == "Node" else
                {"name": name, "namespace": ns}}
        if kind == "Node":
            if any(ps.node == name for ps in self.pods.values()):
                raise NotImplementedError(f"deleting node {name} with pods bound to it")
            before = len(self.nodes)
            self.nodes = [n for n in self.nodes if n.name != name]
            if len(self.nodes) == before:
                raise ValueError(f"no node {name}")
            self._event({"id": op.id, "delete": {"operation": meta}})
            self._wake(NODE_DELETE)
        else:
            ps = self.pods.pop(f"{ns}/{name}", None)
            if ps is None:
                raise ValueError(f"no pod {ns}/{name}")
            self._event({"id": op.id, "delete": {"operation": meta}})
            if ps.node:
                self._wake(POD_DELETE)

    # ---- the SimulationController: the scheduler until it converges ----
    def _schedule(self) -> None:
        if not any(not ps.node and ps.rejectors is None for ps in self.pods.values()) or not self.nodes:
            return
        states = list(self.pods.values())
        bound = [ps for ps in states if ps.node]
        pending = [ps for ps in states if not ps.node]
        order = bound + pending
        node_index = {n.name: i for i, n in enumerate(self.nodes)}
        sched = F.DebuggableScheduler(self.nodes, [ps.pod for ps in order], self.prof, engine=self.make_engine(),
                                      bound=[(i, node_index[ps.node]) for i, ps in enumerate(bound)],
                                      native_annotations=self.native_annotations)
        index = {id(ps): i for i, ps in enumerate(order)}
        key_of = {id(ps): f"{ps.pod.namespace}/{ps.pod.name}" for ps in order}
        while True:
            ready = [ps for ps in pending if not ps.node and ps.rejectors is None and key_of[id(ps)] in self.pods]
            if not ready:
                return
            heap = [(-ps.pod.priority, ps.ordinal, index[id(ps)]) for ps in ready]
            heapq.heapify(heap)
            while heap:
                _, _, i = heapq.heappop(heap)
                ps = order[i]
                if ps.node or ps.rejectors is not None or key_of[id(ps)] not in self.pods:
                    continue
                npre = len(sched.preemptions)
                cyc = sched.schedule(i)
                ps.attempts += 1
                sched.reflect(i, ps.annotations)
                for pi, nom, victims in sched.preemptions[npre:]:
                    for v in victims:
                        vs = order[v]
                        self.pods.pop(key_of[id(vs)], None)
                        vs.node = ""
                        self._npre += 1
                        self._event({"id": f"preemption-{self._npre}", "delete": {
                            "operation": {"typeMeta": {"kind": "Pod"},
                                          "objectMeta": {"name": vs.pod.name, "namespace": vs.pod.namespace}},
                            "preemptedBy": {"name": ps.pod.name, "namespace": ps.pod.namespace},
                            "nodeName": self.nodes[nom].name}})
                        self._wake(POD_DELETE)
                if cyc.selected >= 0:
                    ps.node = self.nodes[cyc.selected].name
                    self._nsched += 1
                    self._event({"id": f"podscheduled-{self._nsched}", "podScheduled": {
                        "pod": {"name": ps.pod.name, "namespace": ps.pod.namespace}, "nodeName": ps.node}})
                    self._wake(POD_ADD)
                else:
                    ps.rejectors = F.DebuggableScheduler.rejecting_plugins(cyc, sched.enc.workload.pods[i],
                                                                           sched.enc.prefilter_reject.get(i))
                for ps2 in pending:     # pods woken by this cycle's events join activeQ now
                    if not ps2.node and ps2.rejectors is None and key_of[id(ps2)] in self.pods and ps2 is not ps:
                        entry = (-ps2.pod.priority, ps2.ordinal, index[id(ps2)])
                        if entry not in heap:
                            heapq.heappush(heap, entry)

    def run(self, ops: Sequence[Operation]) -> dict:
        done = False
        steps = sorted({op.step for op in ops})
        for step in steps:
            self.major, self.minor = step, 0
            for op in ops:
                if op.step == step:
                    self._apply(op)
                    done = done or op.done
            self._schedule()
            if done:
                break
        return self.result(done)

    def result(self, done: bool) -> dict:
        return {
            "phase": "Succeeded" if done else "Paused",
            "step": {"major": self.major, "minor": self.minor},
            "timeline": self.timeline,
            "pods": {k: {"nodeName": ps.node, "attempts": ps.attempts, "annotations": ps.annotations}
                     for k, ps in sorted(self.pods.items())},
        }


def simulate(doc, profiles: Sequence[P.Profile], make_engine: Callable[[], object], rank: int = 0,
             world: int = 1) -> List[dict]:
    """KEP-184: the same scenario under each profile.  Rank r runs a
    contiguous block of profiles; one all_gather_object returns every
    result to every rank (gloo on CPU, RCCL-backed groups on GPUs)."""
    from .replicas import shard
    ops = load_scenario(doc)
    lo, hi = shard(len(profiles), world, rank)
    mine = [ScenarioRunner(profiles[k], make_engine).run(ops) for k in range(lo, hi)]
    if world == 1:
        return mine
    import torch.distributed as dist
    outs: List = [None] * world
    dist.all_gather_object(outs, mine)
    return [r for block in outs for r in block]
