"""Debuggable-scheduler mirror over the device evaluator.

`DebuggableScheduler` plays the role of the upstream framework + the
simulator's wrapped plugins for the Filter/Score path:

- one `Engine.eval()` per pod replaces the N x F wrapped `Filter` calls and
  N x S wrapped `Score` calls (wrappedplugin.go:523, :420) and the
  `NormalizeScore` calls (:388);
- the device result (filter status words, raw and normalised scores) is
  written into `annotations.ResultStore` exactly as the wrappers would have
  written it: `"passed"` / rejection message per (node, plugin) up to the
  first rejection (store.go:423), raw score + raw*weight (store.go:461),
  normalised*weight overwrite for plugins with ScoreExtensions (store.go:481),
  PreFilter / PreScore statuses with Skip recorded as "" (store.go:522, :537);
- Reserve records the selected node (wrappedplugin.go:622 -> store.go:562) and
  `Engine.commit()` assumes the pod.

`DevicePlugin` shows the per-plugin shape a cgo shim presents to the
framework (Name / Filter / Score / NormalizeScore answering from the per-pod
device result in CycleState).  The Go version of that shim is INTEGRATION.md.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import annotations as A
from . import encoder as E
from . import model as m
from . import native
from . import preemption as PR
from . import profile as P

FS_NOT_EVALUATED = E.FS_NOT_EVALUATED

MSG_UNSCHEDULABLE = "node(s) were unschedulable"
MSG_NODE_NAME = "node(s) didn't match the requested node name"
MSG_NODE_AFFINITY = "node(s) didn't match Pod's node affinity/selector"
MSG_NODE_PORTS = "node(s) didn't have free ports for the requested pod ports"
MSG_NA_CONFLICT = "pod affinity terms conflict"
MSG_PTS = "node(s) didn't match pod topology spread constraints"
MSG_PTS_LABEL = MSG_PTS + " (missing required label)"
MSG_IPA = {1: "node(s) didn't match pod affinity rules",
           2: "node(s) didn't match pod anti-affinity rules",
           3: "node(s) didn't satisfy existing pods anti-affinity rules"}
# volume plugins [upstream v1.32 volumerestrictions ErrReasonReadWriteOncePodConflict,
# volumebinding ErrReason* (FindPodVolumes order), volumezone ErrReasonConflict]
MSG_RWOP = "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode"
MSG_VB = ((E.VB_NODE_CONFLICT, "node(s) had volume node affinity conflict"),
          (E.VB_BIND_CONFLICT, "node(s) didn't find available persistent volumes to bind"),
          (E.VB_PV_NOT_EXIST, "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)"))
MSG_VZ = "node(s) had no available volume zone"


def prefilter_framework_message(plugins: Sequence[str]) -> str:
    """RunPreFilterPlugins' status when the merged PreFilterResults leave no node."""
    if len(plugins) == 1:
        return f"node(s) didn't satisfy plugin {plugins[0]}"
    return f"node(s) didn't satisfy plugin(s) [{' '.join(plugins)}] simultaneously"


def fit_reasons(bits: int, res_names: Sequence[str]) -> List[str]:
    """noderesources.fitsRequest reason order: pods, cpu, memory, ephemeral,
    then scalar resources (Go map order; sorted by column here)."""
    out = []
    if bits & 1:
        out.append("Too many pods")
    names = {0: "cpu", 1: "memory", 2: "ephemeral-storage"}
    for r in range(len(res_names)):
        if bits & (1 << (r + 1)):
            out.append("Insufficient " + names.get(r, res_names[r]))
    return out


class Decoder:
    """Turns status words back into the upstream message strings."""

    def __init__(self, enc: E.Encoder):
        self.enc = enc
        self.cl = enc.cluster
        self.taints = enc.cluster.arrays["taints"]

    def message(self, st: int, node: int) -> str:
        pl = (st & 0xFF) - 1
        reason = st >> 8
        if pl == P.NODE_UNSCHEDULABLE:
            return MSG_UNSCHEDULABLE
        if pl == P.NODE_NAME:
            return MSG_NODE_NAME
        if pl == P.TAINT_TOLERATION:
            t = self.cl.taint_vocab[int(self.taints[reason, node]) - 1]
            return f"node(s) had untolerated taint {{{t.key}: {t.value}}}"
        if pl == P.NODE_AFFINITY:
            return MSG_NODE_AFFINITY
        if pl == P.NODE_PORTS:
            return MSG_NODE_PORTS
        if pl == P.NODE_RESOURCES_FIT:
            return ", ".join(fit_reasons(reason, self.cl.res_names))
        if pl == P.POD_TOPOLOGY_SPREAD:
            return MSG_PTS_LABEL if reason == 1 else MSG_PTS
        if pl == P.INTER_POD_AFFINITY:
            return MSG_IPA[reason]
        if pl == P.VOLUME_RESTRICTIONS:
            return MSG_RWOP
        if pl == P.VOLUME_BINDING:
            return ", ".join(msg for bit, msg in MSG_VB if reason & bit)
        if pl == P.VOLUME_ZONE:
            return MSG_VZ
        raise ValueError(f"unexpected status word {st:#x}")


def status_code(st: int, enc: E.Encoder, pod: int, node: int) -> int:
    """framework.Code of the Filter rejection in status word `st` [upstream
    v1.32 Filter returns, SURVEY.md Appendix A]: the node-static plugins
    (NodeUnschedulable, NodeName, TaintToleration, NodeAffinity), a
    PodTopologySpread missing label and an InterPodAffinity affinity
    mismatch are UnschedulableAndUnresolvable (preemption cannot help);
    NodeResourcesFit is Unschedulable unless a request exceeds the node's
    allocatable outright (the InsufficientResource.Unresolvable flag);
    skew and anti-affinity rejections are Unschedulable."""
    pl = (st & 0xFF) - 1
    reason = st >> 8
    if pl < 0:
        return Status.SUCCESS
    if pl in (P.NODE_UNSCHEDULABLE, P.NODE_NAME, P.TAINT_TOLERATION, P.NODE_AFFINITY, P.VOLUME_BINDING,
              P.VOLUME_ZONE):
        return Status.UNSCHEDULABLE_AND_UNRESOLVABLE
    if pl == P.NODE_RESOURCES_FIT:
        req = enc.workload.pods[pod]["req"]
        alloc = enc.cluster.arrays["alloc"]
        for r in range(len(enc.cluster.res_names)):
            if reason & (1 << (r + 1)) and int(req[r]) > int(alloc[r, node]):
                return Status.UNSCHEDULABLE_AND_UNRESOLVABLE
        return Status.UNSCHEDULABLE
    if pl in (P.POD_TOPOLOGY_SPREAD, P.INTER_POD_AFFINITY):
        return Status.UNSCHEDULABLE_AND_UNRESOLVABLE if reason == 1 else Status.UNSCHEDULABLE
    return Status.UNSCHEDULABLE


@dataclass
class PodCycle:
    """Everything the device computed for one pod (one CycleState)."""
    pod: int
    selected: int
    n_feasible: int
    status: int
    score_skip: int
    fstatus: np.ndarray
    raw: np.ndarray
    norm: np.ndarray
    total: np.ndarray


class DebuggableScheduler:
    """Framework loop + wrapped-plugin recording, with the evaluator on the GPU."""

    def __init__(self, nodes: Sequence[m.Node], pods: Sequence[m.Pod], prof: P.Profile,
                 engine: Optional[native.Engine] = None, bound: Sequence = (), native_annotations: bool = True):
        """`pods` holds every pod that will ever be bound or scheduled;
        `bound` = [(pod_index, node_index)] already running at start.
        `native_annotations`: emit filter/score/finalscore-result with the
        native serialiser (ksg_annotate) instead of per-entry Store writes."""
        self.nodes = list(nodes)
        self.pods = list(pods)
        self.prof = prof
        self.enc = E.Encoder(self.nodes, self.pods, prof, bound_pods=[pi for pi, _ in bound])
        self.engine = engine if engine is not None else native.Engine()
        self.engine.load(self.enc, E.encode_profile(prof, self.enc.cluster.res_names))
        # NodeInfo.Pods per node (pod indices): DefaultPreemption's victims
        self.on_node: List[List[int]] = [[] for _ in self.nodes]
        for pi, ni in bound:
            self.engine.commit(pi, ni)
            self.on_node[ni].append(pi)
        self.preemption_on = "DefaultPreemption" in {n for n, _ in prof.plugins}
        # (preemptor, nominated node, victims) per preemption, in order
        self.preemptions: List[tuple] = []
        # result set of a preemptor's first attempt: the storereflector
        # reflects it onto the pod before the retry is recorded
        self.first_attempt: Dict[int, Dict[str, str]] = {}
        self.store = A.ResultStore(prof.weights())
        self.decoder = Decoder(self.enc)
        self.node_names = self.enc.cluster.node_names
        self.enabled = set(prof.enabled_ids())
        self.names_enabled = {n for n, _ in prof.plugins}
        self.annotator = None
        if native_annotations:
            cl = self.enc.cluster
            self.annotator = native.Annotator(
                cl.node_names, P.PLUGIN_NAMES, cl.res_names,
                [f"{{{t.key}: {t.value}}}" for t in cl.taint_vocab], cl.arrays["taints"])
            self._weights = np.array([self.store.score_plugin_weight.get(n, 0) for n in P.PLUGIN_NAMES], np.int64)
            self._norm_mask = sum(1 << pid for pid in range(len(P.PLUGIN_NAMES)) if P.EXT[pid][4])

    # ---- one cycle --------------------------------------------------------
    def evaluate(self, pi: int) -> PodCycle:
        cap = native.CaptureBuffers(len(self.nodes), 1)
        r = self.engine.eval(pi, cap)
        return PodCycle(pi, r.selected, r.n_feasible, r.status, r.score_skip, cap.fstatus[0], cap.raw[0],
                        cap.norm[0], cap.total[0])

    def schedule_one(self, pi: int, record: bool = True) -> int:
        return self._cycle(pi, record).selected

    def schedule(self, pi: int, record: bool = True) -> PodCycle:
        """One scheduling cycle (with DefaultPreemption and the preemptor's
        retry); returns the final cycle."""
        return self._cycle(pi, record)

    @staticmethod
    def rejecting_plugins(cyc: PodCycle, enc_pod, reject=None) -> set:
        """diagnosis.UnschedulablePlugins of a failed cycle: the plugin of
        every node's first rejection, or the PreFilter plugin that ended the
        cycle (`reject` = Encoder.prefilter_reject's entry; NodeAffinity when
        absent)."""
        w = np.asarray(cyc.fstatus)
        w = w[(w != 0) & (w != FS_NOT_EVALUATED)]
        out = {int(x) for x in np.unique(w & 0xFF) - 1}
        if int(enc_pod["flags"]) & E.POD_FLAG_PREFILTER_REJECT:
            out.add(P.NODE_AFFINITY if reject is None else reject[0])
        return out

    def _cycle(self, pi: int, record: bool) -> PodCycle:
        cyc = self.evaluate(pi)
        nominated, victims = -1, []
        if cyc.n_feasible == 0 and self.preemption_on:
            nominated, victims = self.preempt(pi, cyc)
        if record:
            self.record(cyc, nominated)
        if nominated >= 0:
            # prepareCandidate: delete the victims; then the retry (module
            # docstring of preemption.py, step 6)
            if any(self._rwop_shared(v) for v in victims):
                # the encoded VolumeRestrictions conflict of the claim's
                # other users would go stale (encoder.py VOL_RWOP_CONFLICT)
                raise NotImplementedError("a preemption victim holds a ReadWriteOncePod claim another pod uses")
            for v in victims:
                self.engine.uncommit(v, nominated)
                self.on_node[nominated].remove(v)
            self.preemptions.append((pi, nominated, list(victims)))
            if record:
                pod = self.pods[pi]
                self.first_attempt[pi] = self.store.GetStoredResult(pod.namespace, pod.name) or {}
                self.store.DeleteData(pod.namespace, pod.name)
            cyc = self.evaluate(pi)
            if int(cyc.fstatus[nominated]) == 0:   # evaluateNominatedNode: the only feasible node
                only = np.full_like(cyc.fstatus, FS_NOT_EVALUATED)
                only[nominated] = 0
                cyc = PodCycle(pi, nominated, 1, cyc.status & ~native.ST_SCORED, cyc.score_skip, only,
                               cyc.raw, cyc.norm, cyc.total)
            if record:
                self.record(cyc)
        if cyc.selected >= 0:
            self.engine.commit(pi, cyc.selected)
            self.on_node[cyc.selected].append(pi)
        return cyc

    def _rwop_shared(self, q: int) -> bool:
        """Whether pod q holds a ReadWriteOncePod claim another pod also uses."""
        pod = self.pods[q]
        if not pod.claim_names():
            return False
        return bool(PR.rwop_holders(pod, [(i, 0, o) for i, o in enumerate(self.pods) if i != q]))

    def preempt(self, pi: int, cyc: PodCycle):
        """DefaultPreemption.PostFilter for a pod with no feasible node:
        returns (nominated node or -1, victims most important first).  The
        dry run over the candidate nodes is ksg_preempt_victims."""
        pod = self.pods[pi]
        if pod.preemption_policy == "Never":              # PodEligibleToPreemptOthers
            return -1, []
        potential = PR.potential_nodes(cyc.fstatus, self.enc.workload.pods[pi]["req"],
                                       self.enc.cluster.arrays["alloc"])
        if not potential:
            return -1, []
        # nodes without a lower-priority pod fail SelectVictimsOnNode at once
        lists = []
        for n in potential:
            low = [q for q in self.on_node[n] if self.pods[q].priority < pod.priority]
            if low:
                lists.append((n, sorted(low, key=lambda q: PR.importance_key(self.pods[q]))))
        if not lists:
            return -1, []
        holders = PR.rwop_holders(pod, [(q, n, self.pods[q]) for n, v in enumerate(self.on_node) for q in v])
        if PR.rwop_outcome(pod, holders, self.pods) == -1:
            return -1, []
        if PR.needs_static_verdict(self.prof, pod):
            # SelectVictimsOnNode re-runs every filter: a node-static one
            # ordered after the recorded rejection fails the node whatever
            # is removed (ksg_eval_skipping with the dry run's four skipped)
            cap = native.CaptureBuffers(len(self.nodes), 1)
            self.engine.eval_skipping(pi, PR.static_skip_mask(), cap)
            ok = np.asarray(cap.fstatus[0]) == 0
            lists = [(n, v) for n, v in lists if ok[n]]
            if not lists:
                return -1, []
        off = np.zeros(len(lists) + 1, np.int32)
        off[1:] = np.cumsum([len(v) for _, v in lists])
        vic = np.array([q for _, v in lists for q in v], np.int32)
        fits, flags = self.engine.preempt_victims(pi, [n for n, _ in lists], off, vic)
        # DryRunPreemption from offset 0: the first num_candidates candidates in node order
        want = PR.num_candidates(len(potential), self.prof)
        cands = []
        for k, (n, v) in enumerate(lists):
            chosen = [int(q) for q, f in zip(v, flags[off[k]:off[k + 1]]) if f]
            if fits[k] and chosen:
                cands.append((n, chosen))
                if len(cands) >= want:
                    break
        if not cands:
            return -1, []
        node = PR.pick_one_node([(n, [self.pods[q] for q in v], 0) for n, v in cands])
        return node, dict(cands)[node]

    def run_queue(self, first: int, count: int):
        """Device-resident queue: no per-pod host round trip.  With
        DefaultPreemption enabled, the pods that could find a victim (those
        of higher priority than some pod already placed or placed before
        them) run as single cycles first; the rest go to ksg_run_queue."""
        head = 0
        if self.preemption_on:
            low = min((self.pods[q].priority for v in self.on_node for q in v), default=None)
            for k in range(count):
                pod = self.pods[first + k]
                if PR.may_preempt(pod, low):
                    head = k + 1
                low = pod.priority if low is None else min(low, pod.priority)
        pl = np.zeros(count, np.int32)
        res = np.zeros(count, native.RESULT_DTYPE)
        for k in range(head):
            cyc = self._cycle(first + k, record=False)
            pl[k] = cyc.selected
            res[k] = (cyc.selected, cyc.n_feasible, cyc.status, cyc.score_skip)
        if head < count:
            pl[head:], res[head:] = self.engine.run_queue(first + head, count - head)
            for k in range(head, count):
                if pl[k] >= 0:
                    self.on_node[pl[k]].append(first + k)
        return pl, res

    # ---- recording (what the wrapped plugins write to the Store) ---------
    def record(self, cyc: PodCycle, nominated: int = -1):
        pod = self.pods[cyc.pod]
        rec = self.enc.workload.pods[cyc.pod]
        ns, name = pod.namespace, pod.name
        st = self.store
        fskip = int(rec["filter_skip"])
        if cyc.status & native.ST_IPA_PREFILTER_SKIP:
            fskip |= 1 << P.INTER_POD_AFFINITY
        # PreFilter (wrappedplugin.go:504-512): RunPreFilterPlugins stops at a
        # rejection, or when the merged PreFilterResults leave no node (the
        # plugin that emptied them recorded success and its node names)
        reject = self.enc.prefilter_reject.get(cyc.pod) if rec["flags"] & E.POD_FLAG_PREFILTER_REJECT else None
        names_of = self.enc.prefilter_results.get(cyc.pod, {})
        for pid in self.prof.prefilter_order():
            pname = P.PLUGIN_NAMES[pid]
            if reject is not None and pid == reject[0] and reject[1] is not None:
                st.AddPreFilterResult(ns, name, pname, reject[1])
                break
            st.AddPreFilterResult(ns, name, pname, "" if (fskip >> pid) & 1 else A.SUCCESS, names_of.get(pid))
            if reject is not None and pid == reject[0]:
                break
        # Filter
        order = [p for p in self.prof.filter_order() if not (fskip >> p) & 1]
        if self.annotator is not None:
            return self._record_native(cyc, ns, name, order, nominated)
        evaluated = []
        for n in range(len(self.nodes)):
            s = int(cyc.fstatus[n])
            if s == FS_NOT_EVALUATED:
                continue
            evaluated.append(n)
            node = self.node_names[n]
            fail = (s & 0xFF) - 1
            for pid in order:
                if pid == fail:
                    st.AddFilterResult(ns, name, node, P.PLUGIN_NAMES[pid], self.decoder.message(s, n))
                    break
                st.AddFilterResult(ns, name, node, P.PLUGIN_NAMES[pid], A.PASSED)
        if cyc.n_feasible == 0:
            # DefaultPreemption PostFilter (wrappedplugin.go:562-577): with every
            # pod at equal priority there is never a victim, so nothing is
            # nominated and every explicitly evaluated node gets an empty entry.
            if "DefaultPreemption" in self.names_enabled:
                st.AddPostFilterResult(ns, name, self.node_names[nominated] if nominated >= 0 else "",
                                       "DefaultPreemption", [self.node_names[n] for n in evaluated])
            return
        if cyc.n_feasible >= 2:
            sskip = cyc.score_skip
            for pid in self.prof.prescore_order():
                st.AddPreScoreResult(ns, name, P.PLUGIN_NAMES[pid], "" if (sskip >> pid) & 1 else A.SUCCESS)
            feas = [n for n in range(len(self.nodes)) if cyc.fstatus[n] == 0]
            for pid in self.prof.score_order():
                if (sskip >> pid) & 1:
                    continue
                pname = P.PLUGIN_NAMES[pid]
                for n in feas:
                    st.AddScoreResult(ns, name, self.node_names[n], pname, int(cyc.raw[pid, n]))
                if P.EXT[pid][4]:
                    for n in feas:
                        st.AddNormalizedScoreResult(ns, name, self.node_names[n], pname, int(cyc.norm[pid, n]))
        self._record_bind(cyc, ns, name)

    def _record_native(self, cyc: PodCycle, ns: str, name: str, order: List[int], nominated: int = -1):
        """Filter/Score/NormalizeScore entries serialised in one native call."""
        st = self.store
        score_order: List[int] = []
        if cyc.n_feasible >= 2:
            score_order = [p for p in self.prof.score_order() if not (cyc.score_skip >> p) & 1]
        f, s, t = self.annotator.annotate(order, score_order, self._norm_mask, self._weights, cyc.n_feasible,
                                          cyc.fstatus, cyc.raw, cyc.norm)
        st.AddSerializedResult(ns, name, A.FILTER, f)
        st.AddSerializedResult(ns, name, A.SCORE, s)
        st.AddSerializedResult(ns, name, A.FINALSCORE, t)
        if cyc.n_feasible == 0:
            if "DefaultPreemption" in self.names_enabled:
                evaluated = np.nonzero(cyc.fstatus != FS_NOT_EVALUATED)[0]
                st.AddPostFilterResult(ns, name, self.node_names[nominated] if nominated >= 0 else "",
                                       "DefaultPreemption", [self.node_names[n] for n in evaluated])
            return
        if cyc.n_feasible >= 2:
            for pid in self.prof.prescore_order():
                st.AddPreScoreResult(ns, name, P.PLUGIN_NAMES[pid], "" if (cyc.score_skip >> pid) & 1 else A.SUCCESS)
        self._record_bind(cyc, ns, name)

    def _record_bind(self, cyc: PodCycle, ns: str, name: str):
        st = self.store
        if cyc.selected < 0:
            return
        # Reserve / Permit / PreBind / Bind of the default plugins.
        st.AddSelectedNode(ns, name, self.node_names[cyc.selected])
        if P.VOLUME_BINDING in self.enabled:
            st.AddReserveResult(ns, name, "VolumeBinding", A.SUCCESS)
            st.AddPreBindResult(ns, name, "VolumeBinding", A.SUCCESS)
        if "DefaultBinder" in self.names_enabled:
            st.AddBindResult(ns, name, "DefaultBinder", A.SUCCESS)

    def annotations(self, pi: int) -> Optional[Dict[str, str]]:
        """The stored result of the pod's cycle.  A preemptor has two: the
        first attempt is already reflected onto the pod; the retry is merged
        over it as the reflector's next pass would (with result-history)."""
        pod = self.pods[pi]
        cur = self.store.GetStoredResult(pod.namespace, pod.name)
        if pi not in self.first_attempt:
            return cur
        return A.merged_reflection(A.merged_reflection({}, self.first_attempt[pi]), cur)

    def reflect(self, pi: int, pod_annotations: Dict[str, str]) -> None:
        """storereflector: merge every result set of the pod's last cycle into
        its annotations (history appended, oldest first) and drop the stored
        data, as after the reflector's pod update."""
        pod = self.pods[pi]
        first = self.first_attempt.pop(pi, None)
        if first:
            pod_annotations.update(first)
            A.update_result_history(pod_annotations, first)
        A.reflect(self.store, pod.namespace, pod.name, pod_annotations)


class Status:
    """framework.Status subset: code + reasons (Message joins with ", ")."""
    SUCCESS, ERROR, UNSCHEDULABLE, UNSCHEDULABLE_AND_UNRESOLVABLE, SKIP = 0, 1, 2, 3, 5   # framework.Code

    def __init__(self, code: int = 0, *reasons: str):
        self.code = code
        self.reasons = list(reasons)

    def is_success(self) -> bool:
        return self.code == Status.SUCCESS

    def message(self) -> str:
        return ", ".join(self.reasons)


class DevicePlugin:
    """One in-tree plugin as the framework sees it, answered from the
    device's per-pod result.  `Name()` returns the in-tree name so the
    simulator's wrapper and Store key results exactly as before
    (wrappedplugin.go:406,438,542)."""

    def __init__(self, sched: DebuggableScheduler, pid: int):
        self.s = sched
        self.pid = pid

    def Name(self) -> str:
        return P.PLUGIN_NAMES[self.pid]

    def Filter(self, cyc: PodCycle, node: int) -> Status:
        st = int(cyc.fstatus[node])
        if (st & 0xFF) - 1 == self.pid:
            return Status(status_code(st, self.s.enc, cyc.pod, node), self.s.decoder.message(st, node))
        return Status()

    def PreFilter(self, cyc: PodCycle) -> Status:
        """Skip for plugins whose PreFilter skips this pod (encoder
        filter_skip, InterPodAffinity's from the device); NodeAffinity
        rejects a pod whose matchFields name no node."""
        rec = self.s.enc.workload.pods[cyc.pod]
        reject = self.s.enc.prefilter_reject.get(cyc.pod)
        if int(rec["flags"]) & E.POD_FLAG_PREFILTER_REJECT and reject is not None and reject[0] == self.pid:
            if reject[1] is not None:
                return Status(Status.UNSCHEDULABLE_AND_UNRESOLVABLE, reject[1])
        fskip = int(rec["filter_skip"])
        if cyc.status & native.ST_IPA_PREFILTER_SKIP:
            fskip |= 1 << P.INTER_POD_AFFINITY
        return Status(Status.SKIP) if (fskip >> self.pid) & 1 else Status()

    def PreScore(self, cyc: PodCycle) -> Status:
        return Status(Status.SKIP) if (cyc.score_skip >> self.pid) & 1 else Status()

    def Score(self, cyc: PodCycle, node: int):
        return int(cyc.raw[self.pid, node]), Status()

    def NormalizeScore(self, cyc: PodCycle, scores: Dict[int, int]) -> Status:
        for n in scores:
            scores[n] = int(cyc.norm[self.pid, n])
        return Status()
