"""Shared test helpers: run the same workload through pyoracle (object model),
the C++ oracle and, on a GPU box, the HIP library; compare everything the
wrapped plugins would record."""
import numpy as np

from conftest import pkg

E = pkg("encoder")
P = pkg("profile")
F = pkg("framework")
A = pkg("annotations")
native = pkg("native")


def capture_queue(engine, n_pods, n_nodes):
    cap = native.CaptureBuffers(n_nodes, n_pods)
    pl, res = engine.run_queue(0, n_pods, capture=cap)
    return pl, res, cap


def compare_engine_runs(enc, prof, eng_a, eng_b, label=""):
    """Run the whole queue with capture on two engines; assert bit-exact equality
    of placements, per-node filter status words, and raw / normalised scores of
    every feasible node of every scored pod."""
    pf = E.encode_profile(prof, enc.cluster.res_names)
    eng_a.load(enc, pf)
    eng_b.load(enc, pf)
    n = len(enc.workload.pods)
    N = len(enc.cluster.node_names)
    pa, ra, ca = capture_queue(eng_a, n, N)
    pb, rb, cb = capture_queue(eng_b, n, N)
    np.testing.assert_array_equal(pa, pb, err_msg=f"{label}: placements")
    np.testing.assert_array_equal(ra["n_feasible"], rb["n_feasible"], err_msg=f"{label}: n_feasible")
    np.testing.assert_array_equal(ra["status"], rb["status"], err_msg=f"{label}: status")
    np.testing.assert_array_equal(ra["score_skip"], rb["score_skip"], err_msg=f"{label}: score_skip")
    np.testing.assert_array_equal(ca.fstatus, cb.fstatus, err_msg=f"{label}: filter status words")
    mask = np.asarray(P.Profile().enabled_ids())
    for k in range(n):
        if not (ra["status"][k] & native.ST_SCORED):
            continue
        feas = ca.fstatus[k] == 0
        for pid in range(native.NPLUGINS):
            if not ((prof_mask(pf) >> pid) & 1) or ((int(ra["score_skip"][k]) >> pid) & 1):
                continue
            np.testing.assert_array_equal(ca.raw[k, pid][feas], cb.raw[k, pid][feas],
                                          err_msg=f"{label}: raw pod {k} plugin {P.PLUGIN_NAMES[pid]}")
            np.testing.assert_array_equal(ca.norm[k, pid][feas], cb.norm[k, pid][feas],
                                          err_msg=f"{label}: norm pod {k} plugin {P.PLUGIN_NAMES[pid]}")
        np.testing.assert_array_equal(ca.total[k][feas], cb.total[k][feas], err_msg=f"{label}: total pod {k}")
    return pa


def prof_mask(pf):
    return pf["score_mask"]


def scheduler_annotations(nodes, pods, prof, engine):
    """Drive DebuggableScheduler pod by pod (eval + record + commit) and return
    the per-pod annotation maps."""
    s = F.DebuggableScheduler(nodes, pods, prof, engine=engine)
    out = []
    for i in range(len(pods)):
        s.schedule_one(i)
        out.append(s.annotations(i))
    return out


def pyoracle_annotations(nodes, pods, prof, bound=()):
    """`pods` = the queue; `bound` = [(pod, node name)] already running.
    A preemptor's first attempt is reflected onto the pod before its retry
    is recorded (A.reflect / A.merged_reflection)."""
    import pyoracle
    store = A.ResultStore(prof.weights())
    recs = pyoracle.run_queue(nodes, list(bound), pods, prof)
    names = set(n for n, _ in prof.plugins)

    def put(ns, nm, r):
        for pl, msg in r["prefilter_status"].items():
            store.AddPreFilterResult(ns, nm, pl, msg, r["prefilter_result"].get(pl))
        for node, d in r["filter"].items():
            for pl, msg in d.items():
                store.AddFilterResult(ns, nm, node, pl, msg)
        if r["n_feasible"] == 0:
            if "DefaultPreemption" in names:
                store.AddPostFilterResult(ns, nm, r.get("nominated", ""), "DefaultPreemption", list(r["filter"].keys()))
        for pl, msg in r["prescore"].items():
            store.AddPreScoreResult(ns, nm, pl, msg)
        for node, d in r["score"].items():
            for pl, v in d.items():
                store.AddScoreResult(ns, nm, node, pl, int(v))
        for node, d in r["finalscore"].items():
            for pl, v in d.items():
                w = store.score_plugin_weight.get(pl, 0)
                if w and P.EXT[P.PLUGIN_ID[pl]][4]:
                    store.AddNormalizedScoreResult(ns, nm, node, pl, int(v) // w)
        if r["selected"]:
            store.AddSelectedNode(ns, nm, r["selected"])
            if "VolumeBinding" in names:
                store.AddReserveResult(ns, nm, "VolumeBinding", "success")
                store.AddPreBindResult(ns, nm, "VolumeBinding", "success")
            if "DefaultBinder" in names:
                store.AddBindResult(ns, nm, "DefaultBinder", "success")

    out = []
    for pod, r in zip(pods, recs):
        ns, nm = pod.namespace, pod.name
        if "first_attempt" in r:
            put(ns, nm, r["first_attempt"])
            pod_ann = {}
            A.reflect(store, ns, nm, pod_ann)
            put(ns, nm, r)
            out.append(A.merged_reflection(pod_ann, store.GetStoredResult(ns, nm)))
        else:
            put(ns, nm, r)
            out.append(store.GetStoredResult(ns, nm))
    return out, recs
