"""README known-answer test (README.md:56-81) and the
reference's store contract tests restated (store_test.go)."""
import json

from conftest import pkg

G = pkg("generator")
A = pkg("annotations")
P = pkg("profile")


def test_readme_kat_pyoracle():
    import pyoracle
    nodes, pods, prof = G.readme_kat()
    r = pyoracle.run_queue(nodes, [], pods, prof)[0]
    for node in ("node-282x7", "node-gp9t4"):
        sc, fs = r["score"][node], r["finalscore"][node]
        assert sc["NodeResourcesFit"] == "73" and fs["NodeResourcesFit"] == "73"
        assert sc["NodeResourcesBalancedAllocation"] == "76" and fs["NodeResourcesBalancedAllocation"] == "76"
        assert sc["TaintToleration"] == "0" and fs["TaintToleration"] == "300"
        assert sc["ImageLocality"] == "0" and fs["ImageLocality"] == "0"
        # v1.32: NodeAffinity / PodTopologySpread / InterPodAffinity Skip at PreScore
        for pl in ("NodeAffinity", "PodTopologySpread", "InterPodAffinity"):
            assert pl not in sc
    # deterministic tie-break: lowest node index
    assert r["selected"] == "node-282x7"


def test_readme_kat_oracle_cpp():
    import binding
    E = pkg("encoder")
    native = pkg("native")
    nodes, pods, prof = G.readme_kat()
    enc = E.Encoder(nodes, pods, prof)
    o = binding.Oracle(1)
    o.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    cap = native.CaptureBuffers(2, 1)
    r = o.eval(0, cap)
    assert r.n_feasible == 2 and r.selected == 0
    assert list(cap.raw[0, P.NODE_RESOURCES_FIT]) == [73, 73]
    assert list(cap.raw[0, P.BALANCED_ALLOCATION]) == [76, 76]
    assert list(cap.norm[0, P.TAINT_TOLERATION]) == [100, 100]


# The second reference-held vector (simulator/docs/plugin-extender.md:85-107):
# the same README cluster after one 100m / 16Gi pod went to node-282x7.  Only
# the per-plugin values and the selection are asserted: the plugin set there
# is an older upstream's (AzureDiskLimits, EBSLimits, ...) plus the sample's
# out-of-tree NodeNumber plugin.
KAT2 = {"node-282x7": {"NodeResourcesFit": 47, "NodeResourcesBalancedAllocation": 52},
        "node-gp9t4": {"NodeResourcesFit": 73, "NodeResourcesBalancedAllocation": 76}}
KAT2_SELECTED = "node-gp9t4"


def test_readme_kat2_pyoracle():
    import pyoracle
    nodes, pods, prof = G.readme_kat2()
    first, second = pyoracle.run_queue(nodes, [], pods, prof)[:2]
    assert first["selected"] == "node-282x7"
    for node, want in KAT2.items():
        for pl, v in want.items():
            assert second["score"][node][pl] == str(v)
            assert second["finalscore"][node][pl] == str(v)   # weight 1, no ScoreExtensions
        assert second["finalscore"][node]["TaintToleration"] == "300"
    assert second["selected"] == KAT2_SELECTED


def test_readme_kat2_oracle_cpp():
    import binding
    E = pkg("encoder")
    native = pkg("native")
    nodes, pods, prof = G.readme_kat2()
    enc = E.Encoder(nodes, pods, prof)
    o = binding.Oracle(1)
    o.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    r0 = o.eval(0)
    assert r0.selected == 0
    o.commit(0, r0.selected)
    cap = native.CaptureBuffers(2, 1)
    r = o.eval(1, cap)
    assert r.n_feasible == 2 and enc.cluster.node_names[r.selected] == KAT2_SELECTED
    for n, node in enumerate(enc.cluster.node_names):
        assert cap.raw[0, P.NODE_RESOURCES_FIT, n] == KAT2[node]["NodeResourcesFit"]
        assert cap.raw[0, P.BALANCED_ALLOCATION, n] == KAT2[node]["NodeResourcesBalancedAllocation"]
    # the batched queue of the oracle agrees
    o.load(enc, E.encode_profile(prof, enc.cluster.res_names))
    pl, _ = o.run_queue(0, 2)
    assert [enc.cluster.node_names[x] for x in pl] == ["node-282x7", KAT2_SELECTED]


def test_store_weight_application():
    # store_test.go:284-333: raw "10" with weight 2 -> final "20"
    s = A.ResultStore({"plugin1": 2})
    s.AddScoreResult("default", "pod1", "node1", "plugin1", 10)
    r = s.results["default/pod1"]
    assert r.score == {"node1": {"plugin1": "10"}}
    assert r.finalscore == {"node1": {"plugin1": "20"}}
    # normalised score overwrites the final score (store_test.go:448-540)
    s.AddNormalizedScoreResult("default", "pod1", "node1", "plugin1", 7)
    assert r.finalscore == {"node1": {"plugin1": "14"}}
    # a plugin without a weight entry gets weight 0
    s.AddScoreResult("default", "pod1", "node1", "plugin2", 10)
    assert r.finalscore["node1"]["plugin2"] == "0"


def test_store_get_stored_result_shapes():
    # store_test.go:584-835 "success without some data on store"
    s = A.ResultStore({})
    s.AddFilterResult("default", "pod1", "node0", "plugin1", "passed")
    s.AddFilterResult("default", "pod1", "node1", "plugin1", "passed")
    a = s.GetStoredResult("default", "pod1")
    assert a[A.FILTER] == json.dumps({"node0": {"plugin1": "passed"}, "node1": {"plugin1": "passed"}},
                                     separators=(",", ":"))
    for k in (A.SCORE, A.FINALSCORE, A.POSTFILTER, A.PRESCORE, A.PREFILTER_RESULT, A.PREFILTER_STATUS,
              A.PERMIT, A.PERMIT_TIMEOUT, A.RESERVE, A.PREBIND, A.BIND):
        assert a[k] == "{}"
    assert a[A.SELECTED_NODE] == ""
    assert s.GetStoredResult("default", "nope") is None
    # postfilter: nominated node gets the victim message, others an empty map
    s.AddPostFilterResult("default", "pod2", "node0", "plugin1", ["node0", "node1"])
    assert s.GetStoredResult("default", "pod2")[A.POSTFILTER] == \
        '{"node0":{"plugin1":"preemption victim"},"node1":{}}'


def test_go_json_escaping():
    assert A.go_marshal({"b": "<x>&", "a": "q\"\\\n "}) == \
        '{"a":"q\\"\\\\\\n\\u2028","b":"\\u003cx\\u003e\\u0026"}'
    assert A.go_marshal({"k": ["n1", "n2"]}) == '{"k":["n1","n2"]}'
    assert A.go_marshal({"\x01": "\x1f"}) == '{"\\u0001":"\\u001f"}'
    # bytewise key order
    assert A.go_marshal({"b": "1", "B": "2", "a": "3"}) == '{"B":"2","a":"3","b":"1"}'


def test_result_history_trimming():
    # storereflector_test.go:83-205: history appended, oldest dropped past 256 KiB
    ann = {}
    big = "x" * (100 * 1024)
    for i in range(4):
        A.update_result_history(ann, {"k": big, "i": str(i)})
        hist = json.loads(ann[A.RESULT_HISTORY])
        assert hist[-1]["i"] == str(i)
        assert len(ann[A.RESULT_HISTORY].encode()) <= A.TOTAL_ANNOTATION_SIZE_LIMIT
    assert [h["i"] for h in json.loads(ann[A.RESULT_HISTORY])] == ["2", "3"]


def test_profile_weights_and_order():
    # plugins_test.go:183-203 weights; scheduler_test.go:523-541 order
    prof = P.default_profile()
    w = prof.weights()
    assert w["TaintToleration"] == 3 and w["NodeAffinity"] == 2 and w["NodeResourcesFit"] == 1
    assert w["PodTopologySpread"] == 2 and w["InterPodAffinity"] == 2
    assert w["NodeResourcesBalancedAllocation"] == 1 and w["ImageLocality"] == 1
    assert w["NodeName"] == 1   # weight 0 -> 1 (plugins.go:296-300)
    assert prof.simulator_plugin_names()[4] == "TaintTolerationWrapped"
    assert [P.PLUGIN_NAMES[p] for p in prof.filter_order()] == [
        "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
        "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding", "VolumeZone", "PodTopologySpread",
        "InterPodAffinity"]
