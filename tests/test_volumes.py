"""Pods with persistentVolumeClaim volumes: VolumeRestrictions,
NodeVolumeLimits, VolumeBinding and VolumeZone (tests/zoo.py zoo_volumes;
the reference's export sample case 2 plus a pod claiming pvc1).  Both
restatements (the object-model pyoracle and the C++ oracle over the encoded
volume programs) agree byte for byte; the GPU matches them (-m gpu).  Parity
unpinned against Go: no reference fixture holds a volume plugin's result."""
import json
import os

import pytest

from conftest import pkg
from helpers import pyoracle_annotations

E = pkg("encoder")
F = pkg("framework")
I = pkg("ingest")
m = pkg("model")
P = pkg("profile")
HERE = os.path.dirname(os.path.abspath(__file__))


def _sched_annotations(nodes, pods, prof, engine, bound=()):
    s = F.DebuggableScheduler(nodes, pods, prof, engine=engine, bound=bound)
    done = {pi for pi, _ in bound}
    out = []
    for i in range(len(pods)):
        if i in done:
            continue
        s.schedule_one(i)
        out.append(s.annotations(i))
    return out


def _compare(nodes, pods, prof, engine, bound=()):
    queue = [p for i, p in enumerate(pods) if i not in {pi for pi, _ in bound}]
    want, recs = pyoracle_annotations(nodes, queue, prof, [(pods[pi], nodes[ni].name) for pi, ni in bound])
    got = _sched_annotations(nodes, pods, prof, engine, bound)
    for k, (w, g) in enumerate(zip(want, got)):
        assert w == g, f"queue pod {k} ({queue[k].name}): annotations differ\nwant {w}\ngot  {g}"
    return recs


def export_case2_with_claim():
    """export.md case 2 (bound pvc1 -> pv1, an available pv2) with two nodes
    and pods claiming pvc1, a missing claim, and none."""
    doc = json.load(open(os.path.join(HERE, "golden", "export_md.json")))["case2"]
    doc = json.loads(json.dumps(doc))
    doc["nodes"] = [{"metadata": {"name": f"node-{k}", "labels": {"kubernetes.io/hostname": f"node-{k}"}},
                     "status": {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "110"}}} for k in range(2)]

    def pod(name, claim=None):
        spec = {"containers": [{"name": "c", "image": "nginx", "resources": {"requests": {"cpu": "100m"}}}]}
        if claim is not None:
            spec["volumes"] = [{"name": "data", "persistentVolumeClaim": {"claimName": claim}}]
        return {"metadata": {"name": name, "namespace": "default"}, "spec": spec}
    doc["pods"] = [pod("uses-pvc1", "pvc1"), pod("no-volume"), pod("uses-missing", "nope"), pod("again", "pvc1")]
    # the sample's config without the legacy volume-limit plugins the
    # simulator's registry does not hold (tests/test_ingest.py)
    from test_ingest import export_config_loadable
    doc["schedulerConfig"] = export_config_loadable()
    return doc


def test_export_case2_claim_cpu_oracles():
    import binding
    snap = I.load_snapshot(export_case2_with_claim())
    assert snap.pods[0].storage.pvcs[("default", "pvc1")].fully_bound()
    recs = _compare(snap.nodes, snap.pods, snap.profile, binding.Oracle(2))
    # pvc1 -> pv1 (hostPath, no node affinity): every volume plugin passes;
    # VolumeZone skips (no zone labels); the missing claim ends PreFilter
    assert recs[0]["n_feasible"] == 2
    assert recs[0]["filter"]["node-0"]["VolumeBinding"] == "passed"
    assert "VolumeZone" not in recs[0]["filter"]["node-0"]
    assert recs[2]["prefilter_status"]["VolumeRestrictions"] == 'persistentvolumeclaim "nope" not found'
    assert recs[2]["n_feasible"] == 0 and not recs[2]["filter"]


@pytest.mark.parametrize("seed", range(4))
def test_zoo_volumes_pyoracle_vs_oracle(seed):
    import binding
    from zoo import zoo_volumes
    nodes, pods, prof = zoo_volumes(seed)
    recs = _compare(nodes, pods, prof, binding.Oracle(2))
    msgs = {msg for r in recs for d in r["filter"].values() for msg in d.values()}
    assert any("volume node affinity conflict" in x for x in msgs)
    assert any("no available volume zone" in x for x in msgs)


def test_zoo_volumes_rwop_held_by_running_pods():
    import binding
    from zoo import zoo_volumes
    nodes, pods, prof, run = zoo_volumes(1, bound=True)
    recs = _compare(nodes, pods, prof, binding.Oracle(2), bound=run)
    msgs = {msg for r in recs for d in r["filter"].values() for msg in d.values()}
    assert any("ReadWriteOncePod" in x for x in msgs)


def test_refusals():
    from zoo import zoo_volumes
    nodes, pods, prof = zoo_volumes(0)
    st = pods[0].storage
    # a ReadWriteOncePod claim shared by two queued pods: the first placement decides
    pods[3].volumes = [("v", "persistentVolumeClaim", "rwop-0")]
    pods[4].volumes = [("v", "persistentVolumeClaim", "rwop-0")]
    with pytest.raises(NotImplementedError):
        E.Encoder(nodes, pods, prof)
    pods[4].volumes = []
    E.Encoder(nodes, pods, prof)
    # an unbound WaitForFirstConsumer claim another PV could bind statically
    st.pvs["pv-free"] = m.PersistentVolume("pv-free", storage_class="any")
    st.pvcs[("default", "free")] = m.PersistentVolumeClaim("free", "default", "", "any")
    pods[5].volumes = [("v", "persistentVolumeClaim", "free")]
    with pytest.raises(NotImplementedError):
        E.Encoder(nodes, pods, prof)
    # ephemeral volumes stay refused
    pods[5].volumes = [("v", "ephemeral", "")]
    with pytest.raises(NotImplementedError):
        E.Encoder(nodes, pods, prof)


@pytest.fixture(scope="module")
def gpu(built):
    native = pkg("native")
    eng = native.Engine(device=0)
    yield eng
    eng.close()


@pytest.mark.gpu
def test_export_case2_claim_gpu(gpu):
    snap = I.load_snapshot(export_case2_with_claim())
    _compare(snap.nodes, snap.pods, snap.profile, gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_zoo_volumes_gpu(gpu, seed):
    from zoo import zoo_volumes
    nodes, pods, prof = zoo_volumes(seed)
    _compare(nodes, pods, prof, gpu)


@pytest.mark.gpu
def test_zoo_volumes_rwop_gpu(gpu):
    from zoo import zoo_volumes
    nodes, pods, prof, run = zoo_volumes(1, bound=True)
    _compare(nodes, pods, prof, gpu, bound=run)


@pytest.mark.gpu
def test_zoo_volumes_queue_matches_oracle(gpu):
    """The device-resident queue (ksg_run_queue: pods with claims take the
    queue kernels) against the C++ oracle at a larger size."""
    import binding
    from helpers import compare_engine_runs
    from zoo import zoo_volumes
    nodes, pods, prof = zoo_volumes(5, n_nodes=400, n_pods=600)
    enc = E.Encoder(nodes, pods, prof)
    compare_engine_runs(enc, prof, gpu, binding.Oracle(8), "zoo-volumes-400")
