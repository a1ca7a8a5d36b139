"""Snapshot encoder: cluster objects -> SoA columns + pod programs (include/ksched.h).

This is subsystem (1) of BASELINE.json's north star: NodeInfo/PodInfo become
int64 resource columns, interned uint32 label / taint / image ids and compiled
selector programs, laid out for coalesced reads (column c of node i at
c * n_nodes + i).  Everything string-shaped is resolved here, on the host,
once per workload:

- label keys referenced by any selector or topology key become label columns
  (value id 0 = absent, 1 = "" , 2.. = other values);
- taints become ids of a (key, value, effect) vocabulary; tolerations become
  two bitmaps over that vocabulary per distinct toleration list (all
  tolerations for Filter, the PreferNoSchedule/empty-effect subset for Score,
  taint_toleration.go getAllTolerationPreferNoSchedule [upstream]);
- node affinity / nodeSelector become requirement programs;
- ImageLocality's per-(image) contribution
  `int64(float64(size) * (float64(numNodes) / float64(totalNumNodes)))` is
  node-independent, so it is computed here and the device only tests image
  presence;
- PodTopologySpread / InterPodAffinity label selectors become selector ids; a
  pod's commit program lists the selectors it matches (per-node counts) and the
  affinity-term templates it owns (per-domain tables).

Program grammar (int32 words; offsets are word indices, -1 = absent):
  requirement  := col op nvals vals[nvals]
                  op: 0 In, 1 NotIn, 2 Exists, 3 DoesNotExist, 4 Gt, 5 Lt
                  (Gt/Lt: nvals = 2, vals = lo32 hi32 of the int64 bound), 6 Never
  na_req       := n_sel requirement[n_sel] n_terms (-1 = no required affinity)
                  { n_reqs requirement[n_reqs] }[n_terms]   (n_reqs 0 = empty term)
  na_pref      := n_terms { weight n_reqs requirement[n_reqs] }[n_terms]
  tol          := filter_bits[W] prefer_bits[W],  W = ceil(n_taint_vocab / 32)
  img          := n { image_id+1 contrib_lo contrib_hi }[n]
  node_set     := bits[ceil(n_nodes / 32)]
  pts          := n_hard n_soft require_all
                  { col sel max_skew min_domains self_match na_honor nt_honor }[n_hard]
                  { col sel max_skew na_honor nt_honor is_hostname }[n_soft]
  ipa          := n_aff sel_all self_all col[n_aff]
                  n_anti { col sel }[n_anti]
                  n_pref { col sel weight }[n_pref]          (weight < 0: anti)
                  n_m_anti tmpl[n_m_anti]  n_m_hard tmpl[n_m_hard]  n_m_pref tmpl[n_m_pref]
  commit       := n_sel sel[n_sel] n_tmpl {tmpl weight}[n_tmpl]   (weight: the term's signed
                  preferred weight, 1 for required terms)
  ports        := n_conf conf[n_conf] n_own own[n_own]   (NodePorts: ids into the host-port
                  vocabulary of every (hostIP, protocol, hostPort) any pod uses, sanitised and
                  sorted; conf = the ids HostPortInfo.CheckConflict reports for the pod's ports,
                  own = the pod's ports, which its assume adds to the node's UsedPorts)

A pod's tol..ports programs are contiguous: [blob, blob + blob_len).
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import model as m
from . import profile as P

MAX_RES = 8
NPLUGINS = P.N_PLUGINS
FS_NOT_EVALUATED = 0xFF

OP_IN, OP_NOT_IN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_NEVER = range(7)
_OPS = {m.IN: OP_IN, m.NOT_IN: OP_NOT_IN, m.EXISTS: OP_EXISTS, m.DOES_NOT_EXIST: OP_DNE,
        m.GT: OP_GT, m.LT: OP_LT}

EFFECT_CODE = {m.NO_SCHEDULE: 1, m.PREFER_NO_SCHEDULE: 2, m.NO_EXECUTE: 3}

TMPL_REQ_ANTI, TMPL_REQ_AFF, TMPL_PREF = 0, 1, 2

POD_FLAG_TOL_UNSCHED = 1 << 0
POD_FLAG_NA_REQUIRED = 1 << 1
POD_FLAG_BEST_EFFORT = 1 << 2
POD_FLAG_PREFILTER_REJECT = 1 << 3

VOLUME_PLUGINS = (P.VOLUME_RESTRICTIONS, P.NODE_VOLUME_LIMITS, P.VOLUME_BINDING, P.VOLUME_ZONE)
# the volume program's flag word (_vol) and VolumeBinding's Filter reason bits
VOL_RWOP_CONFLICT = 1 << 0        # VolumeRestrictions rejects every node
VB_NODE_CONFLICT, VB_BIND_CONFLICT, VB_PV_NOT_EXIST = 1, 2, 4
MSG_VB_UNBOUND_IMMEDIATE = "pod has unbound immediate PersistentVolumeClaims"
MSG_NA_CONFLICT = "pod affinity terms conflict"   # NodeAffinity PreFilter (errReasonConflict)

POD_DTYPE = np.dtype([
    ("req", "<i8", (MAX_RES,)), ("nz_cpu", "<i8"), ("nz_mem", "<i8"),
    ("flags", "<u4"), ("filter_skip", "<u4"), ("score_skip", "<u4"),
    ("node_name", "<i4"), ("n_containers", "<i4"), ("tol", "<i4"), ("na_req", "<i4"),
    ("na_pref", "<i4"), ("img", "<i4"), ("node_set", "<i4"), ("pts", "<i4"), ("ipa", "<i4"),
    ("commit", "<i4"), ("blob", "<i4"), ("blob_len", "<i4"), ("ports", "<i4"), ("vol", "<i4"), ("pad", "<i4"),
])
assert POD_DTYPE.itemsize == 152

SYSTEM_DEFAULT_SPREAD = ((3, m.LABEL_HOSTNAME), (5, m.LABEL_ZONE))  # (maxSkew, key), ScheduleAnyway


# ------------------------------------------------------------------ Go math.Log
_LN2HI = 6.93147180369123816490e-01
_LN2LO = 1.90821492927058770002e-10
_L = (6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01,
      2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01,
      1.479819860511658591e-01)


def go_log(x: float) -> float:
    """Port of Go's math.Log (src/math/log.go, FreeBSD e_log.c algorithm).
    Python floats are IEEE-754 doubles with no fused multiply-add, so this
    reproduces Go's float64 result bit for bit."""
    if x != x or x == math.inf:
        return x
    if x < 0:
        return math.nan
    if x == 0:
        return -math.inf
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    L1, L2, L3, L4, L5, L6, L7 = _L
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * _LN2HI - ((hfsq - (s * (hfsq + R) + k * _LN2LO)) - f)


def parse_int64(s: str):
    """strconv.ParseInt(s, 10, 64); None on error."""
    if not s:
        return None
    body = s[1:] if s[0] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        return None
    v = int(s)
    if v < -(1 << 63) or v >= (1 << 63):
        return None
    return v


# ------------------------------------------------------------------ selectors
def canon_selector(ls: Optional[m.LabelSelector], extra: Optional[Dict[str, str]] = None):
    """Canonical, hashable form of metav1.LabelSelectorAsSelector(ls)
    (+ matchLabelKeys merge).  None = labels.Nothing()."""
    if ls is None:
        return None
    reqs = set()
    for k, v in ls.match_labels:
        reqs.add((k, OP_IN, (v,)))
    for r in ls.match_expressions:
        reqs.add((r.key, _OPS[r.operator], tuple(sorted(set(r.values)))))
    if extra:
        for k, v in extra.items():
            reqs.add((k, OP_IN, (v,)))
    return tuple(sorted(reqs))


def selector_matches(canon, labels: Dict[str, str]) -> bool:
    if canon is None:
        return False
    for k, op, vals in canon:
        has = k in labels
        if op == OP_IN:
            if not has or labels[k] not in vals:
                return False
        elif op == OP_NOT_IN:
            if has and labels[k] in vals:
                return False
        elif op == OP_EXISTS:
            if not has:
                return False
        elif op == OP_DNE:
            if has:
                return False
        else:
            return False
    return True


class _PodIndex:
    """Inverted index label (k, v) -> pod ids, to match selectors against
    many pods without a pods x selectors scan."""

    def __init__(self, pods: Sequence[m.Pod]):
        self.pods = pods
        self.by_kv: Dict[Tuple[str, str], List[int]] = defaultdict(list)
        for i, p in enumerate(pods):
            for k, v in p.labels.items():
                self.by_kv[(k, v)].append(i)

    def candidates(self, canon):
        if canon is None:
            return []
        best = None
        for k, op, vals in canon:
            if op == OP_IN:
                c = []
                for v in vals:
                    c.extend(self.by_kv.get((k, v), ()))
                if best is None or len(c) < len(best):
                    best = c
        if best is None:
            return range(len(self.pods))
        return sorted(set(best))

    def matching(self, canon, ns_pred):
        out = []
        for i in self.candidates(canon):
            p = self.pods[i]
            if ns_pred(p) and selector_matches(canon, p.labels):
                out.append(i)
        return out


# ------------------------------------------------------------------ encoded views
class EncodedCluster:
    """Node SoA columns and vocabularies (decode tables for messages)."""

    def __init__(self):
        self.node_names: List[str] = []
        self.res_names: List[str] = []
        self.label_cols: List[str] = []
        self.label_vocab: List[Dict[str, int]] = []
        self.taint_vocab: List[m.Taint] = []
        self.image_vocab: List[str] = []
        self.arrays: Dict[str, np.ndarray] = {}
        self.n_templates = 0
        self.n_selectors = 0


class EncodedWorkload:
    def __init__(self, pods: np.ndarray, prog: np.ndarray, names: List[str]):
        self.pods = pods
        self.prog = prog
        self.names = names          # "namespace/name"


class Encoder:
    """Encodes nodes and every pod that will ever be bound or scheduled."""

    def __init__(self, nodes: Sequence[m.Node], pods: Sequence[m.Pod], prof: P.Profile,
                 bound_pods: Sequence[int] = ()):
        """`bound_pods`: indices of the pods already running when the queue
        starts (they count as users of their claims for VolumeRestrictions)."""
        self.nodes = list(nodes)
        self.pods = list(pods)
        self.prof = prof
        self.bound_pods = set(int(i) for i in bound_pods)
        self.N = len(self.nodes)
        self.node_index = {n.name: i for i, n in enumerate(self.nodes)}
        if len(self.node_index) != self.N:
            raise ValueError("duplicate node names")
        self.prog: List[int] = []
        self._intern_prog: Dict[tuple, int] = {}
        self.max_blob = 0
        # NodeAffinity PreFilterResult.NodeNames per pod (sorted; upstream's
        # sets.UnsortedList order is random)
        self.prefilter_node_names: Dict[int, List[str]] = {}
        # PreFilterResult node names per pod and plugin id (NodeAffinity,
        # VolumeBinding), and the PreFilter that ended a pod's cycle: (plugin
        # id, its status message; None = the plugin returned success with
        # node names, and the framework's merge of the results left none)
        self.prefilter_results: Dict[int, Dict[int, List[str]]] = {}
        self.prefilter_reject: Dict[int, Tuple[int, Optional[str]]] = {}
        self._vol_outcome: Dict[int, dict] = {}   # _volume_plan's PreFilter outcomes, consumed by _encode_pods
        self._build_resources()
        self._build_label_columns()
        self._build_taints()
        self._build_images()
        self._build_topology_universe()
        self._build_ports()
        self.cluster = self._encode_cluster()
        self.workload = self._encode_pods()
        # requirement values may extend a column's vocabulary after the node
        # columns were built; ids stay below col_vocab either way.
        self.cluster.arrays["col_vocab"] = np.array(
            [len(v) + 1 for v in self.label_vocab] or [1], np.int32)

    # -------------------------------------------------------------- resources
    def _build_resources(self):
        scal = set()
        for n in self.nodes:
            scal.update(k for k in n.allocatable if m.is_scalar_resource(k))
        self._req_cache: Dict[int, Tuple[dict, dict]] = {}
        for i, p in enumerate(self.pods):
            r = m.pod_requests(p)
            nz = m.pod_requests(p, non_zero=True)
            self._req_cache[i] = (r, nz)
            scal.update(k for k in r if m.is_scalar_resource(k))
        for name, _ in list(self.prof.fit_resources) + list(self.prof.ba_resources):
            if m.is_scalar_resource(name):
                scal.add(name)
        self.res_names = [m.CPU, m.MEMORY, m.EPHEMERAL] + sorted(scal)
        if len(self.res_names) > MAX_RES:
            raise NotImplementedError(f"more than {MAX_RES} resource columns")
        self.res_col = {r: i for i, r in enumerate(self.res_names)}

    # -------------------------------------------------------------- host ports
    def _build_ports(self):
        """The host-port vocabulary: every sanitised (hostIP, protocol,
        hostPort) a pod of the workload uses, sorted (NodeInfo.UsedPorts only
        ever holds those)."""
        vocab = set()
        for p in self.pods:
            for ip, proto, port in p.host_ports():
                vocab.add((*m.sanitize_host_port(ip, proto), int(port)))
        self.port_vocab = sorted(vocab)
        self.port_id = {t: i for i, t in enumerate(self.port_vocab)}

    def _ports(self, p: m.Pod) -> int:
        want = [(*m.sanitize_host_port(ip, proto), int(port)) for ip, proto, port in p.host_ports()]
        if not want:
            return -1
        conf = set()
        for ip, proto, port in want:   # HostPortInfo.CheckConflict over the vocabulary
            for i, (vip, vproto, vport) in enumerate(self.port_vocab):
                if vproto == proto and vport == port and (
                        ip == m.DEFAULT_BIND_ALL_HOST_IP or vip in (m.DEFAULT_BIND_ALL_HOST_IP, ip)):
                    conf.add(i)
        own = sorted({self.port_id[t] for t in want})
        return self._emit([len(conf)] + sorted(conf) + [len(own)] + own)

    # -------------------------------------------------------------- volumes
    # VolumeRestrictions / NodeVolumeLimits / VolumeBinding / VolumeZone for
    # pods with persistentVolumeClaim volumes [upstream v1.32
    # plugins/volumerestrictions/volume_restrictions.go, nodevolumelimits/
    # csi.go, volumebinding/{volume_binding,binder}.go, volumezone/
    # volume_zone.go; not vendored: parity unpinned, DESIGN.md §9].  PreFilter
    # is decided here, per pod; the per-node Filter predicates go to the
    # device as the pod's volume program (_volume_plan's grammar below).
    def _volume_label_keys(self, p: m.Pod):
        """Node label keys the pod's volume program reads."""
        keys = set()
        st = p.storage
        if not p.claim_names() or st is None:
            return keys
        keys.update(m.VOLUME_ZONE_LABELS)
        for c in p.claim_names():
            pvc = st.claim(p.namespace, c)
            if pvc is None:
                continue
            pv = st.pvs.get(pvc.volume_name) if pvc.volume_name else None
            if pv is not None:
                for t in pv.node_affinity or ():
                    keys.update(r.key for r in t.match_expressions)
            cls = st.classes.get(pvc.storage_class) if pvc.storage_class else None
            if cls is not None:
                for term in cls.allowed_topologies:
                    keys.update(k for k, _ in term)
        return keys

    @staticmethod
    def _label_zones(pv: m.PersistentVolume, value: str):
        """volumehelpers.LabelZonesToSet: "__"-separated, no blank member."""
        zones = [z.strip() for z in value.split("__")]
        if any(not z for z in zones):
            raise NotImplementedError(f"PersistentVolume {pv.name}: zone label {value!r} has an empty member")
        return sorted(set(zones))

    def _volume_plan(self, i: int, p: m.Pod):
        """(PreFilter Skip bits of the four volume plugins, the volume program
        words or None); the plugins' PreFilter outcomes (rejection message,
        VolumeBinding's PreFilterResult node names) go to self._vol_outcome[i]
        for the ordered PreFilter pass in _encode_pods.

        Volume program (word offsets, the pod's blob):
          flags                    VOL_RWOP_CONFLICT
          n_bound, n_bound x [kind, ...]   VolumeBinding checkBoundClaims, in
                                   volume order: kind 0 = the PV does not
                                   exist; kind 1 = nterms, terms (the PV's
                                   required node affinity on labels only:
                                   CheckNodeAffinity's node has no name, so
                                   matchFields never constrain)
          n_prov, n_prov x [sel, nterms, terms]  the unbound
                                   WaitForFirstConsumer claims: sel = node
                                   index of the claim's selected-node
                                   annotation (-1 none, -2 not in the
                                   snapshot); nterms = -1 for a class that
                                   cannot provision (BindConflict
                                   everywhere), else allowedTopologies as In
                                   terms (0 terms: every node)
          zc[4]                    label columns of volumezone.topologyLabels
          n_zone, n_zone x [col, ga_col, n, ids..., n_ga, ids...]
        """
        all_skip = sum(1 << v for v in VOLUME_PLUGINS)
        claims = p.claim_names()
        if not claims:
            return all_skip, None
        st = p.storage or m.Storage()
        ns = p.namespace
        out = {}
        skip = 0
        missing = next((c for c in claims if st.claim(ns, c) is None), None)
        nf = f'persistentvolumeclaim "{missing}" not found'
        flags = 0
        # VolumeRestrictions: needsRestrictionsCheck (a claim) -> readWriteOncePodPVCsForPod
        if missing is not None:
            out[P.VOLUME_RESTRICTIONS] = ("reject", nf)
        else:
            for c in claims:
                if m.READ_WRITE_ONCE_POD not in st.claim(ns, c).access_modes:
                    continue
                others = self._claim_users.get((ns, c), set()) - {i}
                if i not in self.bound_pods and any(u not in self.bound_pods for u in others):
                    raise NotImplementedError(
                        f"pod {ns}/{p.name}: ReadWriteOncePod claim {c!r} is shared with another queued pod "
                        f"(whose placement decides the conflict)")
                if others:   # StorageInfos.IsPVCUsedByPods: a running pod holds it
                    flags |= VOL_RWOP_CONFLICT
        # NodeVolumeLimits: PreFilter runs for claims; its Filter passes while no
        # node publishes CSI attach limits (checked at ingest)
        # VolumeBinding: podHasPVCs, GetPodVolumeClaims, GetEligibleNodes
        bound, prov = [], []
        vb = None
        for c in claims:
            pvc = st.claim(ns, c)
            if pvc is None:
                vb = ("reject", nf)
                break
            if pvc.deleting:
                vb = ("reject", f'persistentvolumeclaim "{c}" is being deleted')
                break
        if vb is None:
            immediate = False
            for c in claims:
                pvc = st.claim(ns, c)
                if pvc.fully_bound():
                    bound.append(pvc)
                    continue
                cls = st.classes.get(pvc.storage_class) if pvc.storage_class else None
                if cls is not None and cls.binding_mode == m.BINDING_WAIT_FOR_FIRST_CONSUMER and not pvc.volume_name:
                    prov.append((pvc, cls))
                else:
                    immediate = True
            if immediate:
                vb = ("reject", MSG_VB_UNBOUND_IMMEDIATE)
        if vb is None:
            eligible = None
            for pvc in bound:   # GetEligibleNodes: local volumes' hostname In values
                pv = st.pvs.get(pvc.volume_name)
                if pv is None:
                    eligible = None
                    break
                names = set()   # util.GetLocalPersistentVolumeNodeNames
                for t in pv.node_affinity or ():
                    tn = None
                    for r in t.match_expressions:
                        if r.key == m.LABEL_HOSTNAME and r.operator == m.IN:
                            tn = set(r.values) if tn is None else tn & set(r.values)
                    names |= tn or set()
                if names:
                    eligible = names if eligible is None else eligible & names
            if eligible is not None:
                vb = ("names", eligible)
            for pvc, cls in prov:
                for pv in st.pvs.values():
                    if pv.storage_class == pvc.storage_class and pv.claim_ref in (None, (ns, pvc.name)):
                        raise NotImplementedError(
                            f"pod {ns}/{p.name}: claim {pvc.name!r} could bind statically to PersistentVolume "
                            f"{pv.name!r} (findMatchingVolumes is not modelled)")
                if i not in self.bound_pods and self._claim_users.get((ns, pvc.name), set()) - {i}:
                    raise NotImplementedError(
                        f"pod {ns}/{p.name}: unbound claim {pvc.name!r} is shared with another pod "
                        f"(its assumed binding is not modelled)")
        if vb is not None:
            out[P.VOLUME_BINDING] = vb
        # VolumeZone: getPVbyPod
        zone = []
        vz = None
        for c in claims:
            if not c:
                vz = ("reject", "PersistentVolumeClaim had no name")
                break
            pvc = st.claim(ns, c)
            if pvc is None:
                vz = ("reject", f'persistentvolumeclaim "{c}" not found')
                break
            if not pvc.volume_name:
                sc = pvc.storage_class
                if not sc:
                    vz = ("reject", "PersistentVolumeClaim had no pv name and storageClass name")
                    break
                cls = st.classes.get(sc)
                if cls is None:
                    vz = ("reject", f'storageclass.storage.k8s.io "{sc}" not found')
                    break
                if cls.binding_mode == m.BINDING_WAIT_FOR_FIRST_CONSUMER:
                    continue
                vz = ("reject", "PersistentVolume had no name")
                break
            pv = st.pvs.get(pvc.volume_name)
            if pv is None:
                vz = ("reject", f'persistentvolume "{pvc.volume_name}" not found')
                break
            for key in m.VOLUME_ZONE_LABELS:
                if key in pv.labels:
                    zone.append((key, self._label_zones(pv, pv.labels[key])))
        if vz is not None:
            out[P.VOLUME_ZONE] = vz
        elif not zone:
            skip |= 1 << P.VOLUME_ZONE
        self._vol_outcome[i] = out
        # ---- the Filter program
        words = [flags, len(bound)]
        for pvc in bound:
            pv = st.pvs.get(pvc.volume_name)
            if pv is None:
                words.append(0)
                continue
            if pv.source in m.PV_SOURCES_MIGRATED:
                raise NotImplementedError(f"PersistentVolume {pv.name}: {pv.source} (CSI translation not modelled)")
            if pv.node_affinity is None:
                words += [1, -1]
                continue
            terms = []
            for t in pv.node_affinity:
                if not t.match_expressions:
                    if t.match_fields:   # fields only: the nameless node matches
                        terms = None
                        break
                    terms.append([0])    # an empty term matches nothing
                    continue
                tw = [len(t.match_expressions)]
                for r in t.match_expressions:
                    tw += self._requirement(r)
                terms.append(tw)
            if terms is None:
                words += [1, -1]
            else:
                words += [1, len(terms)] + [x for tw in terms for x in tw]
        words.append(len(prov))
        for pvc, cls in prov:
            sel_name = pvc.annotations.get(m.ANN_SELECTED_NODE)
            sel = -1 if sel_name is None else self.node_index.get(sel_name, -2)
            if cls.provisioner in ("", m.NOT_SUPPORTED_PROVISIONER):
                words += [sel, -1]
                continue
            words += [sel, len(cls.allowed_topologies)]
            for term in cls.allowed_topologies:
                words.append(len(term))
                for key, vals in term:
                    col = self.col_index[key]
                    ids = sorted({self._value_id(col, v) for v in vals})
                    words += [col, OP_IN, len(ids)] + ids if ids else [0, OP_NEVER, 0]
        words += [self.col_index.get(k, -1) for k in m.VOLUME_ZONE_LABELS]
        words.append(len(zone))
        for key, vals in zone:
            col = self.col_index[key]
            ga = m.GA_LABEL.get(key, key)
            gcol = self.col_index[ga]
            ids = sorted({self._value_id(col, v) for v in vals})
            gids = sorted({self._value_id(gcol, v) for v in vals})
            words += [col, gcol, len(ids)] + ids + [len(gids)] + gids
        return skip, words

    # -------------------------------------------------------------- labels
    def _pts_constraints(self, pod: m.Pod):
        """(hard, soft) lists of (max_skew, key, canon_selector, min_domains,
        na_policy, nt_policy, self_match) as filterTopologySpreadConstraints /
        buildDefaultConstraints [upstream podtopologyspread/common.go] yield."""
        hard, soft = [], []
        if pod.topology_spread_constraints:
            for c in pod.topology_spread_constraints:
                extra = None
                if c.match_label_keys:
                    extra = {k: pod.labels[k] for k in c.match_label_keys if k in pod.labels} or None
                canon = canon_selector(c.label_selector, extra)
                ent = (c.max_skew, c.topology_key, canon,
                       c.min_domains if c.min_domains is not None else 1,
                       c.node_affinity_policy or m.POLICY_HONOR,
                       c.node_taints_policy or m.POLICY_IGNORE)
                if c.when_unsatisfiable == m.DO_NOT_SCHEDULE:
                    hard.append(ent)
                elif c.when_unsatisfiable == m.SCHEDULE_ANYWAY:
                    soft.append(ent)
        elif pod.default_spread_selector is not None:
            # buildDefaultConstraints: the profile's defaults (System: the
            # two ScheduleAnyway constraints; List: defaultConstraints as
            # written), each with the owners' selector
            canon = canon_selector(pod.default_spread_selector)
            if canon:   # selector.Empty() -> no default constraints
                if self.prof.pts_system_defaulted:
                    for skew, key in SYSTEM_DEFAULT_SPREAD:
                        soft.append((skew, key, canon, 1, m.POLICY_HONOR, m.POLICY_IGNORE))
                for c in () if self.prof.pts_system_defaulted else self.prof.pts_default_constraints:
                    ent = (c.max_skew, c.topology_key, canon, c.min_domains if c.min_domains is not None else 1,
                           c.node_affinity_policy or m.POLICY_HONOR, c.node_taints_policy or m.POLICY_IGNORE)
                    (hard if c.when_unsatisfiable == m.DO_NOT_SCHEDULE else soft).append(ent)
        return hard, soft

    def _build_label_columns(self):
        keys = set()
        uses_name_field = False
        self._pts_cache = {}
        for i, p in enumerate(self.pods):
            if p.node_selector:
                keys.update(p.node_selector)
            for t in (p.node_affinity_required or []):
                keys.update(r.key for r in t.match_expressions)
                uses_name_field |= bool(t.match_fields)
            for pt in (p.node_affinity_preferred or []):
                keys.update(r.key for r in pt.preference.match_expressions)
                uses_name_field |= bool(pt.preference.match_fields)
            hard, soft = self._pts_constraints(p)
            self._pts_cache[i] = (hard, soft)
            keys.update(c[1] for c in hard + soft)
            for t in p.pod_affinity_required + p.pod_anti_affinity_required:
                keys.add(t.topology_key)
            for w in p.pod_affinity_preferred + p.pod_anti_affinity_preferred:
                keys.add(w.term.topology_key)
            keys.update(self._volume_label_keys(p))
        self.label_cols = sorted(keys)
        if uses_name_field:
            self.label_cols.append(m.OBJECT_NAME_FIELD)
        self.col_index = {k: i for i, k in enumerate(self.label_cols)}
        self.label_vocab: List[Dict[str, int]] = [{"": 1} for _ in self.label_cols]
        L, N = len(self.label_cols), self.N
        self.label_val = np.zeros((max(L, 1), N), np.uint32)
        self.label_num = np.zeros((max(L, 1), N), np.int64)
        self.label_num_ok = np.zeros((max(L, 1), N), np.uint8)
        for c, key in enumerate(self.label_cols):
            voc = self.label_vocab[c]
            for i, n in enumerate(self.nodes):
                if key == m.OBJECT_NAME_FIELD:
                    v = n.name
                elif key in n.labels:
                    v = n.labels[key]
                else:
                    continue
                vid = voc.setdefault(v, len(voc) + 1)
                self.label_val[c, i] = vid
                num = parse_int64(v)
                if num is not None:
                    self.label_num[c, i] = num
                    self.label_num_ok[c, i] = 1
        self.has_labels = np.array([1 if n.labels else 0 for n in self.nodes], np.uint8)

    def _value_id(self, col: int, v: str) -> int:
        voc = self.label_vocab[col]
        return voc.setdefault(v, len(voc) + 1)

    # -------------------------------------------------------------- taints
    def _build_taints(self):
        voc: Dict[m.Taint, int] = {}
        for n in self.nodes:
            for t in n.taints:
                if t not in voc:
                    voc[t] = len(voc)
        self.taint_vocab = list(voc)
        self.taint_id = voc
        self.max_taints = max([len(n.taints) for n in self.nodes] + [1])
        taints = np.zeros((self.max_taints, self.N), np.uint32)
        for i, n in enumerate(self.nodes):
            for s, t in enumerate(n.taints):
                taints[s, i] = voc[t] + 1
        self.taints = taints
        self.taint_effect = np.array([EFFECT_CODE.get(t.effect, 0) for t in self.taint_vocab] or [0], np.uint8)
        self.tol_words = max(1, (len(self.taint_vocab) + 31) // 32)

    # -------------------------------------------------------------- images
    def _build_images(self):
        first: Dict[str, int] = {}
        nodes_with: Dict[str, set] = defaultdict(set)
        for n in self.nodes:
            for img in n.images:
                for name in img.names:
                    if name not in first:
                        first[name] = img.size_bytes
                    nodes_with[name].add(n.name)
        self.image_vocab = sorted(first)
        self.image_id = {nm: i for i, nm in enumerate(self.image_vocab)}
        self.image_state = {nm: (first[nm], len(nodes_with[nm])) for nm in first}
        per_node = []
        for n in self.nodes:
            ids = sorted({self.image_id[name] for img in n.images for name in img.names})
            per_node.append(ids)
        self.max_images = max([len(x) for x in per_node] + [1])
        arr = np.zeros((self.max_images, self.N), np.uint32)
        for i, ids in enumerate(per_node):
            for s, iid in enumerate(ids):
                arr[s, i] = iid + 1
        self.images = arr

    # -------------------------------------------------------------- PTS / IPA universe
    @staticmethod
    def _term_scope(t: m.PodAffinityTerm, owner: m.Pod):
        """(canon selector, namespaces, all-namespaces) of framework.AffinityTerm."""
        if t.namespace_selector is not None and not t.namespace_selector.empty():
            raise NotImplementedError("namespaceSelector with requirements is not modelled")
        ns_all = t.namespace_selector is not None
        ns = tuple(sorted(set(t.namespaces)))
        if not t.namespaces and t.namespace_selector is None:
            ns = (owner.namespace,)
        return (canon_selector(t.label_selector), ns, ns_all)

    def _build_topology_universe(self):
        pods = self.pods
        idx = _PodIndex(pods)
        self.pts_sel: Dict[tuple, int] = {}      # (canon, namespace) -> id
        self.ipa_sel: Dict[tuple, int] = {}      # tuple of scopes (conjunction) -> id
        self.templates: Dict[tuple, int] = {}    # (kind, scope, col) -> id; weights ride in commit programs
        self.owned_templates: Dict[int, List[int]] = defaultdict(list)
        for i, p in enumerate(pods):
            hard, soft = self._pts_cache[i]
            for c in hard + soft:
                if c[2] is not None and c[2] != ():
                    self.pts_sel.setdefault((c[2], p.namespace), len(self.pts_sel))
            if p.pod_affinity_required:
                conj = tuple(self._term_scope(t, p) for t in p.pod_affinity_required)
                self.ipa_sel.setdefault(conj, len(self.ipa_sel))
            for t in p.pod_anti_affinity_required:
                self.ipa_sel.setdefault((self._term_scope(t, p),), len(self.ipa_sel))
            for w in p.pod_affinity_preferred + p.pod_anti_affinity_preferred:
                self.ipa_sel.setdefault((self._term_scope(w.term, p),), len(self.ipa_sel))
            # templates owned by p (its terms as an *existing* pod)
            for kind, terms in ((TMPL_REQ_ANTI, [(t, 1) for t in p.pod_anti_affinity_required]),
                                (TMPL_REQ_AFF, [(t, 1) for t in p.pod_affinity_required]),
                                (TMPL_PREF, [(w.term, w.weight) for w in p.pod_affinity_preferred]
                                 + [(w.term, -w.weight) for w in p.pod_anti_affinity_preferred])):
                for t, wt in terms:
                    # one template per (kind, scope, topology key): terms that differ only
                    # in weight share its domain table (each assume adds its own weight),
                    # so an incoming pod looks up one table instead of one per weight
                    key = (kind, self._term_scope(t, p), self.col_index[t.topology_key])
                    tid = self.templates.setdefault(key, len(self.templates))
                    self.owned_templates[i].append((tid, wt))
        n_pts = len(self.pts_sel)
        # selector ids: PTS selectors first, then IPA selectors
        self.ipa_sel = {k: n_pts + v for k, v in self.ipa_sel.items()}
        self.n_selectors = n_pts + len(self.ipa_sel)
        # which pods match which selector (commit programs)
        self.pod_selectors: Dict[int, List[int]] = defaultdict(list)
        for (canon, ns), sid in self.pts_sel.items():
            for j in idx.matching(canon, lambda q, ns=ns: q.namespace == ns and not q.terminating):
                self.pod_selectors[j].append(sid)
        for conj, sid in self.ipa_sel.items():
            cand = None
            for (canon, ns, ns_all) in conj:
                mt = set(idx.matching(canon, lambda q, ns=ns, ns_all=ns_all: ns_all or q.namespace in ns))
                cand = mt if cand is None else cand & mt
            for j in sorted(cand or ()):
                self.pod_selectors[j].append(sid)
        # which templates match which (incoming) pod
        self.pod_tmpl_match: Dict[int, Tuple[List[int], List[int], List[int]]] = defaultdict(lambda: ([], [], []))
        for (kind, (canon, ns, ns_all), col), tid in sorted(self.templates.items(), key=lambda kv: kv[1]):
            for j in idx.matching(canon, lambda q, ns=ns, ns_all=ns_all: ns_all or q.namespace in ns):
                self.pod_tmpl_match[j][kind].append(tid)
        self.tmpl_col = np.zeros(max(len(self.templates), 1), np.int32)
        self.tmpl_kind = np.zeros(max(len(self.templates), 1), np.int32)
        self.tmpl_weight = np.zeros(max(len(self.templates), 1), np.int32)
        for (kind, _, col), tid in self.templates.items():
            self.tmpl_col[tid] = col
            self.tmpl_kind[tid] = kind
            self.tmpl_weight[tid] = 1   # unused: per-term weights are in the owners' commit programs

    # -------------------------------------------------------------- programs
    def _emit(self, words: Sequence[int], intern: bool = False) -> int:
        # Programs are emitted per pod, back to back, so that a pod's programs
        # form one contiguous blob the kernel stages into LDS (ksg_pod.blob).
        key = tuple(words)
        if intern and key in self._intern_prog:
            return self._intern_prog[key]
        off = len(self.prog)
        self.prog.extend(int(w) for w in words)
        if intern:
            self._intern_prog[key] = off
        return off

    def _requirement(self, r: m.Requirement, field: bool = False) -> List[int]:
        if field:
            if r.key != m.OBJECT_NAME_FIELD or r.operator not in (m.IN, m.NOT_IN) or len(r.values) != 1:
                return [0, OP_NEVER, 0]
            col = self.col_index[m.OBJECT_NAME_FIELD]
        else:
            col = self.col_index[r.key]
        op = _OPS.get(r.operator)
        if op is None:
            return [0, OP_NEVER, 0]
        if op in (OP_IN, OP_NOT_IN):
            if not r.values:
                return [0, OP_NEVER, 0]
            ids = sorted({self._value_id(col, v) for v in r.values})
            return [col, op, len(ids)] + ids
        if op in (OP_EXISTS, OP_DNE):
            if r.values:
                return [0, OP_NEVER, 0]
            return [col, op, 0]
        if len(r.values) != 1 or parse_int64(r.values[0]) is None:
            return [0, OP_NEVER, 0]
        v = parse_int64(r.values[0]) & 0xFFFFFFFFFFFFFFFF
        return [col, op, 2, _s32(v & 0xFFFFFFFF), _s32(v >> 32)]

    def _term(self, t: m.NodeSelectorTerm) -> List[int]:
        reqs = [self._requirement(r) for r in t.match_expressions]
        reqs += [self._requirement(r, field=True) for r in t.match_fields]
        out = [len(reqs)]
        for r in reqs:
            out += r
        return out

    def _na_req(self, p: m.Pod) -> int:
        words = []
        sel = sorted((p.node_selector or {}).items())
        words.append(len(sel))
        for k, v in sel:
            col = self.col_index[k]
            words += [col, OP_IN, 1, self._value_id(col, v)]
        if p.node_affinity_required is None:
            words.append(-1)
        else:
            words.append(len(p.node_affinity_required))
            for t in p.node_affinity_required:
                words += self._term(t)
        return self._emit(words)

    def _na_pref(self, p: m.Pod) -> int:
        terms = [pt for pt in p.node_affinity_preferred
                 if pt.weight != 0 and (pt.preference.match_expressions or pt.preference.match_fields)]
        words = [len(terms)]
        for pt in terms:
            words.append(pt.weight)
            words += self._term(pt.preference)
        return self._emit(words)

    def _tol(self, p: m.Pod) -> int:
        W = self.tol_words
        fb = [0] * W
        pb = [0] * W
        pref = [t for t in p.tolerations if t.effect in ("", m.PREFER_NO_SCHEDULE)]
        for v, taint in enumerate(self.taint_vocab):
            if m.tolerations_tolerate(p.tolerations, taint):
                fb[v // 32] |= 1 << (v % 32)
            if m.tolerations_tolerate(pref, taint):
                pb[v // 32] |= 1 << (v % 32)
        return self._emit([_s32(x) for x in fb + pb])

    def _img(self, p: m.Pod) -> int:
        ents = []
        total = self.N
        for c in list(p.init_containers) + list(p.containers):
            name = m.normalized_image_name(c.image)
            if name in self.image_state:
                size, num = self.image_state[name]
                contrib = int(float(size) * (float(num) / float(total)))
                u = contrib & 0xFFFFFFFFFFFFFFFF
                ents += [self.image_id[name] + 1, _s32(u & 0xFFFFFFFF), _s32(u >> 32)]
        return self._emit([len(ents) // 3] + ents)

    def _node_set(self, names) -> int:
        W = (self.N + 31) // 32
        bits = [0] * W
        for nm in names:
            i = self.node_index.get(nm)
            if i is not None:
                bits[i // 32] |= 1 << (i % 32)
        return self._emit([_s32(x) for x in bits], intern=False)

    def _pts(self, i: int, p: m.Pod) -> int:
        hard, soft = self._pts_cache[i]
        if not hard and not soft:
            return -1
        require_all = 1 if (p.topology_spread_constraints or not self.prof.pts_system_defaulted) else 0
        words = [len(hard), len(soft), require_all]

        def sel_of(canon):
            if canon is None or canon == ():
                return -1      # labels.Nothing() or selector.Empty(): counts are 0
            return self.pts_sel[(canon, p.namespace)]

        for skew, key, canon, mind, nap, ntp in hard:
            self_match = 1 if (canon is not None and selector_matches(canon, p.labels)) else 0
            words += [self.col_index[key], sel_of(canon), skew, mind, self_match,
                      int(nap == m.POLICY_HONOR), int(ntp == m.POLICY_HONOR)]
        for skew, key, canon, mind, nap, ntp in soft:
            words += [self.col_index[key], sel_of(canon), skew, int(nap == m.POLICY_HONOR),
                      int(ntp == m.POLICY_HONOR), int(key == m.LABEL_HOSTNAME)]
        return self._emit(words)

    def _ipa(self, i: int, p: m.Pod) -> int:
        ma, mh, mp = self.pod_tmpl_match.get(i, ([], [], []))
        if not (p.pod_affinity_required or p.pod_anti_affinity_required or p.pod_affinity_preferred
                or p.pod_anti_affinity_preferred or ma or mh or mp):
            return -1
        words = []
        if p.pod_affinity_required:
            scopes = tuple(self._term_scope(t, p) for t in p.pod_affinity_required)
            self_all = all(
                (ns_all or p.namespace in ns) and selector_matches(canon, p.labels)
                for (canon, ns, ns_all) in scopes)
            words += [len(p.pod_affinity_required), self.ipa_sel[scopes], int(self_all)]
            words += [self.col_index[t.topology_key] for t in p.pod_affinity_required]
        else:
            words += [0, -1, 0]
        words.append(len(p.pod_anti_affinity_required))
        for t in p.pod_anti_affinity_required:
            words += [self.col_index[t.topology_key], self.ipa_sel[(self._term_scope(t, p),)]]
        prefs = [(w.term, w.weight) for w in p.pod_affinity_preferred] + \
                [(w.term, -w.weight) for w in p.pod_anti_affinity_preferred]
        words.append(len(prefs))
        for t, wt in prefs:
            words += [self.col_index[t.topology_key], self.ipa_sel[(self._term_scope(t, p),)], wt]
        for lst in (ma, mh, mp):
            words.append(len(lst))
            words += lst
        return self._emit(words)

    def _commit(self, i: int) -> int:
        sels = sorted(self.pod_selectors.get(i, []))
        tm = self.owned_templates.get(i, [])
        if not sels and not tm:
            return -1
        return self._emit([len(sels)] + sels + [len(tm)] + [x for pair in tm for x in pair])

    # -------------------------------------------------------------- encode
    def _encode_cluster(self) -> EncodedCluster:
        N, R = self.N, len(self.res_names)
        ec = EncodedCluster()
        ec.node_names = [n.name for n in self.nodes]
        ec.res_names = list(self.res_names)
        ec.label_cols = list(self.label_cols)
        ec.label_vocab = self.label_vocab
        ec.taint_vocab = list(self.taint_vocab)
        ec.image_vocab = list(self.image_vocab)
        alloc = np.zeros((R, N), np.int64)
        for i, n in enumerate(self.nodes):
            for r, q in n.allocatable.items():
                if r in self.res_col:
                    alloc[self.res_col[r], i] = q
        a = ec.arrays
        a["alloc"] = alloc
        a["requested"] = np.zeros((R, N), np.int64)
        a["nonzero"] = np.zeros((2, N), np.int64)
        a["allowed_pods"] = np.array([n.allocatable.get(m.PODS, 0) for n in self.nodes], np.int32)
        a["pod_count"] = np.zeros(N, np.int32)
        a["unschedulable"] = np.array([1 if n.unschedulable else 0 for n in self.nodes], np.uint8)
        a["label_val"] = self.label_val
        a["label_num"] = self.label_num
        a["label_num_ok"] = self.label_num_ok
        a["taints"] = self.taints
        a["taint_effect"] = self.taint_effect
        a["images"] = self.images
        a["has_labels"] = self.has_labels
        L = len(self.label_cols)
        col_vocab = np.array([len(v) + 1 for v in self.label_vocab] or [1], np.int32)
        col_unique = np.zeros(max(L, 1), np.uint8)
        for c in range(L):
            vals = self.label_val[c]
            present = vals[vals != 0]
            col_unique[c] = 1 if len(np.unique(present)) == len(present) else 0
        a["col_vocab"] = col_vocab
        a["col_unique"] = col_unique
        a["tmpl_col"] = self.tmpl_col
        a["tmpl_kind"] = self.tmpl_kind
        a["tmpl_weight"] = self.tmpl_weight
        a["log_table"] = np.array([go_log(float(i)) for i in range(N + 3)], np.float64)
        ec.n_templates = len(self.templates)
        ec.n_selectors = self.n_selectors
        ec.max_taints = self.max_taints
        ec.max_images = self.max_images
        ec.n_images = len(self.image_vocab)
        ec.n_port_vocab = len(self.port_vocab)
        return ec

    def _encode_pods(self) -> EncodedWorkload:
        prof = self.prof
        vol_run = set(VOLUME_PLUGINS) & (set(prof.prefilter_order()) | set(prof.filter_order()))
        if vol_run:
            for p in self.pods:
                bad = p.volumes_needing_plugins()
                if bad:
                    raise NotImplementedError(
                        f"pod {p.namespace}/{p.name}: volume {bad[0][0]!r} ({bad[0][1]}) makes the volume plugins' "
                        f"PreFilter run; of the volume sources only persistentVolumeClaim is modelled")
        self._claim_users: Dict[Tuple[str, str], set] = {}
        for i, p in enumerate(self.pods):
            for c in p.claim_names():
                self._claim_users.setdefault((p.namespace, c), set()).add(i)
        rec = np.zeros(len(self.pods), POD_DTYPE)
        names = []
        ba_cols = [self.res_col[r] for r, _ in prof.ba_resources if r in self.res_col]
        for i, p in enumerate(self.pods):
            names.append(f"{p.namespace}/{p.name}")
            r, nz = self._req_cache[i]
            e = rec[i]
            for k, v in r.items():
                if k in self.res_col:
                    e["req"][self.res_col[k]] = v
            e["nz_cpu"] = nz.get(m.CPU, 0)
            e["nz_mem"] = nz.get(m.MEMORY, 0)
            flags = 0
            if m.tolerations_tolerate(p.tolerations, m.Taint(m.TAINT_NODE_UNSCHEDULABLE, "", m.NO_SCHEDULE)):
                flags |= POD_FLAG_TOL_UNSCHED
            na_required = p.node_selector is not None or p.node_affinity_required is not None
            if na_required:
                flags |= POD_FLAG_NA_REQUIRED
            if all(r.get(self.res_names[c], 0) == 0 for c in ba_cols):
                flags |= POD_FLAG_BEST_EFFORT
            fskip = 0
            sskip = 0
            if not na_required:
                fskip |= 1 << P.NODE_AFFINITY
            if not p.host_ports():
                fskip |= 1 << P.NODE_PORTS     # nodeports PreFilter: Skip without host ports
            vskip, vol_words = self._volume_plan(i, p) if vol_run else (sum(1 << v for v in VOLUME_PLUGINS), None)
            fskip |= vskip   # PreFilter Skip of the volume plugins (all four for a pod without claims)
            hard, soft = self._pts_cache[i]
            if not hard:
                fskip |= 1 << P.POD_TOPOLOGY_SPREAD
            if not soft:
                sskip |= 1 << P.POD_TOPOLOGY_SPREAD
            if p.node_affinity_preferred is None:
                sskip |= 1 << P.NODE_AFFINITY
            sskip |= 1 << P.VOLUME_BINDING
            if prof.ba_skip_best_effort and (flags & POD_FLAG_BEST_EFFORT):
                sskip |= 1 << P.BALANCED_ALLOCATION
            has_pref_pod_aff = bool(p.pod_affinity_preferred or p.pod_anti_affinity_preferred)
            if prof.ignore_preferred_terms_of_existing_pods and not has_pref_pod_aff:
                sskip |= 1 << P.INTER_POD_AFFINITY
            # PreFilter outcomes in the profile's PreFilter order (RunPreFilterPlugins):
            # the first rejection ends the cycle; PreFilterResults merge by
            # intersection, and an empty merge ends it too (framework message)
            outcome = dict(self._vol_outcome.pop(i, {}))
            # NodeAffinity PreFilter: matchFields metadata.name In -> PreFilterResult
            if p.node_affinity_required:
                names_u = None
                all_named = True
                for term in p.node_affinity_required:
                    tn = None
                    for rq in term.match_fields:
                        if rq.key == m.OBJECT_NAME_FIELD and rq.operator == m.IN:
                            s = set(rq.values)
                            tn = s if tn is None else tn & s
                    if tn is None:
                        all_named = False
                        break
                    names_u = tn if names_u is None else names_u | tn
                if all_named and names_u is not None:
                    outcome[P.NODE_AFFINITY] = ("reject", MSG_NA_CONFLICT) if not names_u else ("names", names_u)
            e["node_set"] = -1
            merged = None
            for pid in prof.prefilter_order():
                kind, val = outcome.get(pid, ("ok", None))
                if kind == "reject":
                    flags |= POD_FLAG_PREFILTER_REJECT
                    self.prefilter_reject[i] = (pid, val)
                    break
                if kind == "names":
                    self.prefilter_results.setdefault(i, {})[pid] = sorted(val)
                    if pid == P.NODE_AFFINITY:
                        self.prefilter_node_names[i] = sorted(val)
                    merged = set(val) if merged is None else merged & set(val)
                    if not merged:
                        flags |= POD_FLAG_PREFILTER_REJECT
                        self.prefilter_reject[i] = (pid, None)
                        break
            if merged and not flags & POD_FLAG_PREFILTER_REJECT:
                e["node_set"] = self._node_set(merged)
            e["flags"] = flags
            e["filter_skip"] = fskip
            e["score_skip"] = sskip
            if p.node_name:
                e["node_name"] = self.node_index.get(p.node_name, -2)
            else:
                e["node_name"] = -1
            e["n_containers"] = len(p.containers) + len(p.init_containers)
            blob = len(self.prog)
            e["tol"] = self._tol(p)
            e["na_req"] = self._na_req(p) if na_required else -1
            e["na_pref"] = self._na_pref(p) if p.node_affinity_preferred is not None else -1
            e["img"] = self._img(p)
            e["pts"] = self._pts(i, p)
            e["ipa"] = self._ipa(i, p)
            e["commit"] = self._commit(i)
            e["ports"] = self._ports(p)
            e["vol"] = self._emit(vol_words) if vol_words is not None else -1
            e["blob"] = blob
            e["blob_len"] = len(self.prog) - blob
            self.max_blob = max(self.max_blob, len(self.prog) - blob)
        prog = np.array(self.prog or [0], np.int32)
        return EncodedWorkload(rec, prog, names)


def _s32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def encode_profile(prof: P.Profile, res_names: Sequence[str]) -> dict:
    """KubeSchedulerProfile -> ksg_profile field values."""
    res_col = {r: i for i, r in enumerate(res_names)}
    order = prof.filter_order()
    weights = prof.selection_weights()
    score_mask = 0
    w = [0] * NPLUGINS
    for pid in prof.score_order():
        score_mask |= 1 << pid
        w[pid] = weights.get(P.PLUGIN_NAMES[pid], 1)
    fit = [(res_col[r], wt) for r, wt in prof.fit_resources if r in res_col]
    ba = [res_col[r] for r, _ in prof.ba_resources if r in res_col]
    ign = 0
    for r in res_names:
        if "/" in r and (r in prof.fit_ignored_resources or r.split("/")[0] in prof.fit_ignored_resource_groups):
            ign |= 1 << res_col[r]
    flags = (1 if prof.ba_skip_best_effort else 0) | (2 if prof.ignore_preferred_terms_of_existing_pods else 0)
    prof.validate_args()
    shape = list(prof.fit_shape) if prof.fit_strategy == P.REQUESTED_TO_CAPACITY_RATIO else []
    pad = [0] * (P.MAX_SHAPE - len(shape))
    return dict(n_filter=len(order), filter_order=order + [0] * (NPLUGINS - len(order)),
                score_mask=score_mask, weight=w, fit_strategy=prof.fit_strategy,
                fit_n=len(fit), fit_res=[c for c, _ in fit] + [0] * (MAX_RES - len(fit)),
                fit_w=[wt for _, wt in fit] + [0] * (MAX_RES - len(fit)),
                ba_n=len(ba), ba_res=ba + [0] * (MAX_RES - len(ba)),
                hard_pod_affinity_weight=prof.hard_pod_affinity_weight, flags=flags,
                fit_ignored_res=ign, shape_n=len(shape), shape_util=[u for u, _ in shape] + pad,
                shape_score=[sc * (100 // P.MAX_CUSTOM_PRIORITY_SCORE) for _, sc in shape] + pad)
