"""Result store mirror and annotation serialiser.

Host-side restatement of the debuggable scheduler's output contract:
- `ResultStore` mirrors `resultstore.Store` (simulator/scheduler/plugin/
  resultstore/store.go:19-24): per-pod maps filled through the same Add*
  methods (store.go:423-572), score weights applied by `applyWeightOnScore`
  (store.go:504-507), annotations produced by `GetStoredResult`
  (store.go:133-198) as Go `json.Marshal` output;
- `update_result_history` mirrors storereflector.updateResultHistory
  (simulator/scheduler/storereflector/storereflector.go:163-190), including
  the oldest-first trimming to the 256 KiB annotation budget.

`go_marshal` reproduces encoding/json (Go 1.24) byte for byte for the value
shapes the store emits: map keys sorted bytewise, HTML-safe escaping of <, >
and &, U+2028/U+2029 escaped, invalid UTF-8 replaced by U+FFFD.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional

PREFIX = "kube-scheduler-simulator.sigs.k8s.io/"
PREFILTER_STATUS = PREFIX + "prefilter-result-status"
PREFILTER_RESULT = PREFIX + "prefilter-result"
FILTER = PREFIX + "filter-result"
POSTFILTER = PREFIX + "postfilter-result"
PRESCORE = PREFIX + "prescore-result"
SCORE = PREFIX + "score-result"
FINALSCORE = PREFIX + "finalscore-result"
RESERVE = PREFIX + "reserve-result"
PERMIT = PREFIX + "permit-result"
PERMIT_TIMEOUT = PREFIX + "permit-result-timeout"
PREBIND = PREFIX + "prebind-result"
BIND = PREFIX + "bind-result"
SELECTED_NODE = PREFIX + "selected-node"
RESULT_HISTORY = PREFIX + "result-history"      # storereflector/annotation.go:4

PASSED = "passed"                    # store.go:28
SUCCESS = "success"                  # store.go:30
WAIT = "wait"                        # store.go:32
POSTFILTER_NOMINATED = "preemption victim"   # store.go:34

TOTAL_ANNOTATION_SIZE_LIMIT = 256 * 1024      # apimachinery validation.TotalAnnotationSizeLimitB

_ESC = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t", "\b": "\\b", "\f": "\\f",
        "<": "\\u003c", ">": "\\u003e", "&": "\\u0026", "\u2028": "\\u2028", "\u2029": "\\u2029"}


def go_string(s) -> str:
    """encoding/json encodeState.string with escapeHTML=true."""
    if isinstance(s, bytes):
        s = s.decode("utf-8", errors="replace")
    out = ['"']
    for ch in s:
        e = _ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ord(ch) < 0x20:
            out.append("\\u%04x" % ord(ch))
        elif 0xD800 <= ord(ch) <= 0xDFFF:   # lone surrogate = invalid UTF-8 in Go
            out.append("�")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _sort_key(k: str):
    return k.encode("utf-8", errors="surrogatepass")


def go_marshal(v) -> str:
    """json.Marshal for nil/str/int/list/dict values as the store produces them."""
    if v is None:
        return "null"
    if isinstance(v, str):
        return go_string(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(go_marshal(x) for x in v) + "]"
    if isinstance(v, dict):
        items = sorted(v.items(), key=lambda kv: _sort_key(kv[0]))
        return "{" + ",".join(go_string(k) + ":" + go_marshal(x) for k, x in items) + "}"
    raise TypeError(type(v))


class _PodResult:
    """resultstore.result (store.go:37-90)."""
    __slots__ = ("selected_node", "prescore", "score", "finalscore", "prefilter_status",
                 "prefilter_result", "filter", "postfilter", "permit", "permit_timeout",
                 "reserve", "prebind", "bind", "custom", "serialized")

    def __init__(self):
        self.selected_node = ""
        self.prescore: Dict[str, str] = {}
        self.score: Dict[str, Dict[str, str]] = {}
        self.finalscore: Dict[str, Dict[str, str]] = {}
        self.prefilter_status: Dict[str, str] = {}
        self.prefilter_result: Dict[str, List[str]] = {}
        self.filter: Dict[str, Dict[str, str]] = {}
        self.postfilter: Dict[str, Dict[str, str]] = {}
        self.permit: Dict[str, str] = {}
        self.permit_timeout: Dict[str, str] = {}
        self.reserve: Dict[str, str] = {}
        self.prebind: Dict[str, str] = {}
        self.bind: Dict[str, str] = {}
        self.custom: Dict[str, str] = {}
        self.serialized: Dict[str, str] = {}   # annotation key -> JSON emitted by the native serialiser


class ResultStore:
    """Mirror of resultstore.Store with the same method names and semantics."""

    def __init__(self, score_plugin_weight: Dict[str, int]):
        self.results: Dict[str, _PodResult] = {}
        self.score_plugin_weight = dict(score_plugin_weight)

    def _get(self, namespace: str, pod: str) -> _PodResult:
        k = namespace + "/" + pod
        r = self.results.get(k)
        if r is None:
            r = self.results[k] = _PodResult()
        return r

    # store.go:423
    def AddFilterResult(self, namespace, pod, node, plugin, reason):
        self._get(namespace, pod).filter.setdefault(node, {})[plugin] = reason

    # store.go:442
    def AddPostFilterResult(self, namespace, pod, nominated, plugin, node_names):
        r = self._get(namespace, pod)
        for nm in node_names:
            d = r.postfilter.setdefault(nm, {})
            if nm == nominated:
                d[plugin] = POSTFILTER_NOMINATED

    # store.go:461
    def AddScoreResult(self, namespace, pod, node, plugin, score: int):
        r = self._get(namespace, pod)
        r.score.setdefault(node, {})[plugin] = str(int(score))
        self._add_normalized(r, node, plugin, score)

    # store.go:481
    def AddNormalizedScoreResult(self, namespace, pod, node, plugin, score: int):
        self._add_normalized(self._get(namespace, pod), node, plugin, score)

    def _add_normalized(self, r: _PodResult, node, plugin, score):
        # applyWeightOnScore (store.go:504-507): a plugin missing from the
        # weight map has weight 0.
        w = self.score_plugin_weight.get(plugin, 0)
        r.finalscore.setdefault(node, {})[plugin] = str(int(score) * w)

    # store.go:522
    def AddPreFilterResult(self, namespace, pod, plugin, reason, node_names: Optional[List[str]] = None):
        r = self._get(namespace, pod)
        r.prefilter_status[plugin] = reason
        if node_names is not None:
            r.prefilter_result[plugin] = list(node_names)

    # store.go:537
    def AddPreScoreResult(self, namespace, pod, plugin, reason):
        self._get(namespace, pod).prescore[plugin] = reason

    def AddPermitResult(self, namespace, pod, plugin, status, timeout: str):
        r = self._get(namespace, pod)
        r.permit[plugin] = status
        r.permit_timeout[plugin] = timeout

    # store.go:562
    def AddSelectedNode(self, namespace, pod, node):
        self._get(namespace, pod).selected_node = node

    def AddReserveResult(self, namespace, pod, plugin, status):
        self._get(namespace, pod).reserve[plugin] = status

    def AddBindResult(self, namespace, pod, plugin, status):
        self._get(namespace, pod).bind[plugin] = status

    def AddPreBindResult(self, namespace, pod, plugin, status):
        self._get(namespace, pod).prebind[plugin] = status

    def AddCustomResult(self, namespace, pod, key, result):
        self._get(namespace, pod).custom[key] = result

    def AddSerializedResult(self, namespace, pod, key, value: str):
        """Annotation value already serialised from the capture SoA
        (native.Annotator, byte-identical to marshalling the map)."""
        self._get(namespace, pod).serialized[key] = value

    def DeleteData(self, namespace, pod):
        self.results.pop(namespace + "/" + pod, None)

    # store.go:133-198
    def GetStoredResult(self, namespace: str, pod: str) -> Optional[Dict[str, str]]:
        r = self.results.get(namespace + "/" + pod)
        if r is None:
            return None
        a = {
            PREFILTER_RESULT: go_marshal(r.prefilter_result),
            PREFILTER_STATUS: go_marshal(r.prefilter_status),
            FILTER: go_marshal(r.filter),
            POSTFILTER: go_marshal(r.postfilter),
            PRESCORE: go_marshal(r.prescore),
            SCORE: go_marshal(r.score),
            FINALSCORE: go_marshal(r.finalscore),
            RESERVE: go_marshal(r.reserve),
            PERMIT_TIMEOUT: go_marshal(r.permit_timeout),
            PERMIT: go_marshal(r.permit),
            PREBIND: go_marshal(r.prebind),
            BIND: go_marshal(r.bind),
        }
        a.update(r.serialized)
        for k, v in r.custom.items():
            a.setdefault(k, v)
        a[SELECTED_NODE] = r.selected_node
        return a


def update_result_history(pod_annotations: Dict[str, str], result_set: Dict[str, str]) -> None:
    """storereflector.updateResultHistory: append `result_set` to the JSON
    history annotation, dropping the oldest entries until it fits."""
    prev = pod_annotations.get(RESULT_HISTORY, "[]")
    results = json.loads(prev)
    results.append(dict(result_set))
    while results:
        enc = go_marshal(results)
        if len(enc.encode("utf-8")) <= TOTAL_ANNOTATION_SIZE_LIMIT:
            pod_annotations[RESULT_HISTORY] = enc
            return
        results = results[1:]
    raise ValueError("result history still exceeds annotation limit even after removing several histories")


def reflect(store: ResultStore, namespace: str, pod: str, pod_annotations: Dict[str, str]) -> bool:
    """storeAllResultToPodFunc (storereflector.go:87-161) minus the API round
    trip: merge the stored results into the pod's annotations, append the
    history entry and drop the stored data."""
    m = store.GetStoredResult(namespace, pod)
    if not m:
        return False
    pod_annotations.update(m)
    update_result_history(pod_annotations, m)
    store.DeleteData(namespace, pod)
    return True


def merged_reflection(pod_annotations: Dict[str, str], result_set: Optional[Dict[str, str]]) -> Dict[str, str]:
    """The pod's annotations after one more reflection of `result_set`
    (storeAllResultToPodFunc), without touching the inputs."""
    out = dict(pod_annotations)
    if result_set:
        out.update(result_set)
        update_result_history(out, result_set)
    return out
