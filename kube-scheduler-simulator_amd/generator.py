"""Seeded synthetic clusters and pod queues (numpy PCG64).

C1 (seed 1): 100 nodes x 1,000 pods, default profile, Z=4, no taints, 20 % nodeSelector.
C2 (seed 2): 5,000 x 50,000, Fit(LeastAllocated) + BA + Taint + NodeAffinity;
             10 % nodes NoSchedule dedicated=<pool>, 10 % PreferNoSchedule spot=true;
             30 % pods tolerate; 25 % required zone affinity; 25 % preferred
             instance-type affinity (weights 1-100).
C3 (seed 3): 15,000 x 150,000, Z=16, 500 apps (Zipf 1.2); every pod: PTS {zone
             maxSkew 5 ScheduleAnyway, hostname maxSkew 1 DoNotSchedule}; 30 %
             preferred anti-affinity hostname(same app); 10 % required affinity
             zone(other app).
C4 (seed 4): R what-if replicas of the C2 cluster/queue; per replica weights in
             [1,5] per score plugin and strategy in {LeastAllocated, MostAllocated}
             drawn from seed 4+r.
C5 (seed 5): 100,000 nodes; amd.com/gpu on 30 % of nodes, 10 % pods request 1-8;
             64 taints/node from a 1,024-entry vocabulary (>= 95 % PreferNoSchedule);
             10,000 images (10 MiB-2 GiB log-uniform), 50 per node Zipf(1.1); pods
             with 1-3 containers over the same vocabulary.

Every config can be scaled down (n_nodes / n_pods) for parity tests.
"""
from __future__ import annotations

import functools
from typing import List, Optional, Tuple

import numpy as np

from . import model as m
from . import profile as P

GI = 1024 ** 3
MI = 1024 ** 2
CPU_CHOICES = [100, 250, 500, 1000, 2000, 4000]
MEM_CHOICES = [128 * MI * (2 ** k) for k in range(7)]   # 128Mi .. 8Gi
INSTANCE_TYPES = [f"m{k}.{s}" for k in (5, 6) for s in ("large", "xlarge", "2xlarge", "4xlarge")]
POOLS = [f"pool-{k:02d}" for k in range(32)]


def _node(i: int, rng, zones: int, extra_alloc=None) -> m.Node:
    z = i % zones
    labels = {
        m.LABEL_HOSTNAME: f"node-{i:06d}",
        m.LABEL_ZONE: f"zone-{z}",
        m.LABEL_REGION: f"region-{z // 4}",
        "node.kubernetes.io/instance-type": INSTANCE_TYPES[int(rng.integers(len(INSTANCE_TYPES)))],
        "pool": POOLS[int(rng.integers(len(POOLS)))],
    }
    alloc = {
        m.CPU: int(rng.choice([16, 32, 64, 96])) * 1000,
        m.MEMORY: int(rng.choice([64, 128, 256, 512])) * GI,
        m.EPHEMERAL: 200 * GI,
        m.PODS: 110,
    }
    if extra_alloc:
        alloc.update(extra_alloc)
    return m.Node(name=f"node-{i:06d}", labels=labels, allocatable=alloc)


def _pod(j: int, rng, best_effort_frac=0.05, image: str = "registry.k8s.io/pause:3.10") -> m.Pod:
    if rng.random() < best_effort_frac:
        req = {}
    else:
        req = {m.CPU: int(rng.choice(CPU_CHOICES)), m.MEMORY: int(rng.choice(MEM_CHOICES))}
    return m.Pod(name=f"pod-{j:06d}", containers=[m.Container(image=image, requests=req)])


def config1(n_nodes: int = 100, n_pods: int = 1000, seed: int = 1):
    rng = np.random.Generator(np.random.PCG64(seed))
    Z = 4
    nodes = [_node(i, rng, Z) for i in range(n_nodes)]
    pods = []
    for j in range(n_pods):
        p = _pod(j, rng)
        if rng.random() < 0.20:
            p.node_selector = {m.LABEL_ZONE: f"zone-{int(rng.integers(Z))}"}
        pods.append(p)
    return nodes, pods, P.default_profile()


def config2(n_nodes: int = 5000, n_pods: int = 50000, seed: int = 2, zones: int = 8):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = [_node(i, rng, zones) for i in range(n_nodes)]
    for n in nodes:
        u = rng.random()
        if u < 0.10:
            n.taints.append(m.Taint("dedicated", n.labels["pool"], m.NO_SCHEDULE))
        elif u < 0.20:
            n.taints.append(m.Taint("spot", "true", m.PREFER_NO_SCHEDULE))
    pods = []
    for j in range(n_pods):
        p = _pod(j, rng)
        if rng.random() < 0.30:
            if rng.random() < 0.5:
                p.tolerations = [m.Toleration("dedicated", m.OP_EQUAL, POOLS[int(rng.integers(len(POOLS)))],
                                              m.NO_SCHEDULE)]
            else:
                p.tolerations = [m.Toleration("spot", m.OP_EXISTS, "", ""),
                                 m.Toleration("dedicated", m.OP_EXISTS, "", m.NO_SCHEDULE)]
        if rng.random() < 0.25:
            k = int(rng.integers(1, 4))
            zs = tuple(sorted({f"zone-{int(z)}" for z in rng.integers(0, zones, size=k)}))
            p.node_affinity_required = [m.NodeSelectorTerm(
                match_expressions=(m.Requirement(m.LABEL_ZONE, m.IN, zs),))]
        if rng.random() < 0.25:
            it = INSTANCE_TYPES[int(rng.integers(len(INSTANCE_TYPES)))]
            p.node_affinity_preferred = [m.PreferredSchedulingTerm(
                int(rng.integers(1, 101)),
                m.NodeSelectorTerm(match_expressions=(
                    m.Requirement("node.kubernetes.io/instance-type", m.IN, (it,)),)))]
        pods.append(p)
    return nodes, pods, P.config2_profile()


def kubelet_memory(nodes, pods, seed: int = 12, pod_frac: float = 0.3):
    """Memory as real clusters report it: node allocatable = capacity minus
    kube-reserved / system-reserved / the eviction threshold, a whole number of
    Ki but not of Mi (kubelet's status.allocatable, e.g. "65544720Ki"), and a
    share of the pods requesting decimal quantities ("300M", "1500M": 10^6-byte
    multiples).  Outside the 32-bit MiB forms; the wide-memory instance of the
    speculate-and-verify walk covers it."""
    rng = np.random.Generator(np.random.PCG64(seed))
    for n in nodes:
        reserved_ki = int(rng.integers(256 * 1024, 2 * 1024 * 1024)) | 1   # odd Ki: never whole MiB
        n.allocatable[m.MEMORY] = n.allocatable[m.MEMORY] - reserved_ki * 1024
    for p in pods:
        if rng.random() < pod_frac:
            for c in p.containers:
                if c.requests.get(m.MEMORY):
                    c.requests[m.MEMORY] = int(rng.integers(1, 80)) * 100 * 1000 * 1000   # 100M .. 7900M
    return nodes, pods


def config2_kubelet(n_nodes: int = 5000, n_pods: int = 50000, seed: int = 2):
    """configs[1] with kubelet-style memory (kubelet_memory)."""
    nodes, pods, prof = config2(n_nodes, n_pods, seed)
    kubelet_memory(nodes, pods)
    return nodes, pods, prof


@functools.lru_cache(maxsize=None)
def _zipf_cdf(n: int, a: float) -> np.ndarray:
    w = 1.0 / np.arange(1, n + 1) ** a
    w /= w.sum()
    # Generator.choice(n, size, p=w) draws exactly this way (cdf of p,
    # normalised by its last entry, searched with one uniform per sample);
    # the cdf is built once per (n, a) instead of once per call.
    cdf = w.cumsum()
    cdf /= cdf[-1]
    cdf.setflags(write=False)
    return cdf


def _zipf_choice(rng, n: int, a: float, size: int):
    return _zipf_cdf(n, a).searchsorted(rng.random(size), side="right").astype(np.int64)


def config3(n_nodes: int = 15000, n_pods: int = 150000, seed: int = 3, zones: int = 16, apps: int = 500):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = [_node(i, rng, zones) for i in range(n_nodes)]
    app_of = _zipf_choice(rng, apps, 1.2, n_pods)
    pods = []
    for j in range(n_pods):
        p = _pod(j, rng)
        a = int(app_of[j])
        p.labels = {"app": f"app-{a:03d}"}
        sel = m.LabelSelector(match_labels=(("app", f"app-{a:03d}"),))
        p.topology_spread_constraints = [
            m.TopologySpreadConstraint(5, m.LABEL_ZONE, m.SCHEDULE_ANYWAY, sel),
            m.TopologySpreadConstraint(1, m.LABEL_HOSTNAME, m.DO_NOT_SCHEDULE, sel),
        ]
        if rng.random() < 0.30:
            p.pod_anti_affinity_preferred = [m.WeightedPodAffinityTerm(
                int(rng.integers(1, 101)), m.PodAffinityTerm(sel, m.LABEL_HOSTNAME))]
        if rng.random() < 0.10:
            b = int(rng.integers(apps))
            if b == a:
                b = (b + 1) % apps
            osel = m.LabelSelector(match_labels=(("app", f"app-{b:03d}"),))
            p.pod_affinity_required = [m.PodAffinityTerm(osel, m.LABEL_ZONE)]
        pods.append(p)
    return nodes, pods, P.config3_profile()


def replica_profiles(n_replicas: int, seed: int = 4) -> List[P.Profile]:
    """C4: per-replica weights in [1,5] per score plugin and Fit strategy."""
    out = []
    for r in range(n_replicas):
        rng = np.random.Generator(np.random.PCG64(seed + r))
        w = {k: int(rng.integers(1, 6)) for k in
             ("TaintToleration", "NodeAffinity", "NodeResourcesFit", "NodeResourcesBalancedAllocation")}
        strat = P.LEAST_ALLOCATED if rng.random() < 0.5 else P.MOST_ALLOCATED
        out.append(P.config2_profile(strategy=strat, weights=w))
    return out


def default_replica_profiles(n_replicas: int, seed: int = 6) -> List[P.Profile]:
    """What-if replicas of the in-tree default profile (the headline's
    multi-GPU ranks): every Score plugin's weight in [1, 5] and the Fit
    strategy drawn per replica; replica 0 is the default profile itself."""
    out = [P.default_profile()]
    for r in range(1, n_replicas):
        rng = np.random.Generator(np.random.PCG64(seed + r))
        prof = P.default_profile()
        prof.plugins = [(n, int(rng.integers(1, 6)) if w else 0) for n, w in prof.plugins]
        prof.fit_strategy = P.LEAST_ALLOCATED if rng.random() < 0.5 else P.MOST_ALLOCATED
        out.append(prof)
    return out


def config4(n_replicas: int = 1024, n_nodes: int = 5000, n_pods: int = 50000):
    nodes, pods, base = config2(n_nodes, n_pods, seed=2)
    return nodes, pods, base, replica_profiles(n_replicas)


def config5(n_nodes: int = 100000, n_pods: int = 100000, seed: int = 5, n_images: int = 10000,
            taint_vocab: int = 1024, taints_per_node: int = 64, images_per_node: int = 50):
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = np.exp(rng.uniform(np.log(10 * MI), np.log(2 * GI), size=n_images)).astype(np.int64)
    img_names = [f"registry.example.com/img-{k:05d}:v1" for k in range(n_images)]
    vocab = []
    for k in range(taint_vocab):
        eff = m.PREFER_NO_SCHEDULE if rng.random() < 0.97 else m.NO_SCHEDULE
        vocab.append(m.Taint(f"t{k % 97}.example.com/k{k}", f"v{k % 13}", eff))
    nodes = []
    for i in range(n_nodes):
        extra = {"amd.com/gpu": int(rng.choice([4, 8]))} if rng.random() < 0.30 else None
        n = _node(i, rng, 16, extra)
        ts = rng.choice(taint_vocab, size=taints_per_node, replace=False)
        n.taints = [vocab[int(t)] for t in ts]
        ims = np.unique(_zipf_choice(rng, n_images, 1.1, images_per_node))
        n.images = [m.ImageState((img_names[int(k)],), int(sizes[int(k)])) for k in ims]
        nodes.append(n)
    pods = []
    for j in range(n_pods):
        nc = int(rng.integers(1, 4))
        conts = []
        for c in range(nc):
            req = {m.CPU: int(rng.choice(CPU_CHOICES)), m.MEMORY: int(rng.choice(MEM_CHOICES))}
            if c == 0 and rng.random() < 0.10:
                req["amd.com/gpu"] = int(rng.integers(1, 9))
            conts.append(m.Container(image=img_names[int(_zipf_choice(rng, n_images, 1.1, 1)[0])],
                                     requests=req))
        p = m.Pod(name=f"pod-{j:06d}", containers=conts)
        k = int(rng.integers(0, 8))
        p.tolerations = [m.Toleration(vocab[int(t)].key, m.OP_EXISTS) for t in
                         rng.choice(taint_vocab, size=k, replace=False)]
        pods.append(p)
    prof = P.Profile(plugins=[("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0),
                              ("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
                              ("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1),
                              ("DefaultBinder", 0)],
                     fit_resources=[(m.CPU, 1), (m.MEMORY, 1), ("amd.com/gpu", 1)])
    return nodes, pods, prof


def readme_kat() -> Tuple[List[m.Node], List[m.Pod], P.Profile]:
    """The README.md:56-81 example: two template nodes (4 CPU / 32Gi / 110 pods,
    web/components/lib/templates/node.yaml:6-13) and a pause:3.5 pod requesting
    100m / 16Gi (web/components/lib/templates/pod.yaml:8-15)."""
    nodes = [m.Node(name=nm, labels={m.LABEL_HOSTNAME: nm},
                    allocatable={m.CPU: 4000, m.MEMORY: 32 * GI, m.PODS: 110})
             for nm in ("node-282x7", "node-gp9t4")]
    pod = m.Pod(name="hoge-pod", containers=[m.Container(
        image="registry.k8s.io/pause:3.5", requests={m.CPU: 100, m.MEMORY: 16 * GI})])
    return nodes, [pod], P.default_profile()


def readme_kat2() -> Tuple[List[m.Node], List[m.Pod], P.Profile]:
    """The second reference-held vector (simulator/docs/plugin-extender.md:
    85-107): the README cluster after one 100m / 16Gi pod went to node-282x7;
    the next identical pod sees node-282x7 at NodeResourcesFit 47 /
    BalancedAllocation 52 (assume: NonZeroRequested feeds Fit, Requested
    feeds BalancedAllocation, whose memory fraction is capped at exactly 1),
    node-gp9t4 at 73 / 76, and is placed on node-gp9t4.  As a queue: the
    first pod lands on node-282x7 (lowest-index tie-break of two equal
    nodes), the second is the documented one."""
    nodes, pods, prof = readme_kat()
    second = m.Pod(name="pod-8ldq5", containers=[m.Container(
        image="registry.k8s.io/pause:3.5", requests={m.CPU: 100, m.MEMORY: 16 * GI})])
    return nodes, pods + [second], prof


def preemption_case(n_nodes: int = 40, n_bound: int = 160, n_queue: int = 120, seed: int = 7):
    """A cluster filled with lower-priority running pods and a queue of
    higher-priority pods that only fit by preemption (DefaultPreemption
    parity cases).  Small nodes (4-8 cores, 8-16 GiB, 6-12 pods) so that
    both "Insufficient" and "Too many pods" rejections are preemptable; 10 %
    of nodes NoSchedule-tainted (unresolvable, never candidates); 5 %
    of queued pods preemptionPolicy Never; running pods' start times spread
    over an hour, some unset.  Returns (nodes, pods, bound [(pod, node)],
    profile); pods = running pods, then the queue in PrioritySort order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = []
    for i in range(n_nodes):
        nd = _node(i, rng, 4)
        nd.allocatable[m.CPU] = int(rng.choice([4, 6, 8])) * 1000
        nd.allocatable[m.MEMORY] = int(rng.choice([8, 12, 16])) * GI
        nd.allocatable[m.PODS] = int(rng.integers(6, 13))
        if rng.random() < 0.10:
            nd.taints = [m.Taint("dedicated", "infra", m.NO_SCHEDULE)]
        nodes.append(nd)
    t0 = 1_700_000_000 * 10 ** 9
    pods, bound = [], []
    free = [[nd.allocatable[m.CPU], nd.allocatable[m.MEMORY], nd.allocatable[m.PODS]] for nd in nodes]
    for j in range(n_bound):
        p = m.Pod(name=f"run-{j:05d}", containers=[m.Container(
            image="registry.k8s.io/pause:3.10",
            requests={m.CPU: int(rng.choice([250, 500, 1000, 1500])), m.MEMORY: int(rng.choice([1, 2, 3])) * GI})])
        p.priority = int(rng.choice([0, 10, 10, 100, 500]))
        p.start_time = None if rng.random() < 0.15 else t0 + int(rng.integers(0, 3600)) * 10 ** 9
        ok = [i for i in range(n_nodes) if not nodes[i].taints and free[i][0] >= p.containers[0].requests[m.CPU]
              and free[i][1] >= p.containers[0].requests[m.MEMORY] and free[i][2] >= 1]
        if not ok:
            continue
        i = ok[int(rng.integers(len(ok)))]
        free[i][0] -= p.containers[0].requests[m.CPU]
        free[i][1] -= p.containers[0].requests[m.MEMORY]
        free[i][2] -= 1
        p.node_name = nodes[i].name
        bound.append((len(pods), i))
        pods.append(p)
    queue = []
    for j in range(n_queue):
        p = _pod(j, rng, best_effort_frac=0.05)
        if p.containers[0].requests:
            p.containers[0].requests[m.CPU] = int(rng.choice([500, 1000, 2000, 3000]))
            p.containers[0].requests[m.MEMORY] = int(rng.choice([1, 2, 4, 6])) * GI
        p.priority = int(rng.choice([0, 10, 50, 200, 200, 1000]))
        if rng.random() < 0.05:
            p.preemption_policy = "Never"
        queue.append(p)
    queue.sort(key=lambda p: -p.priority)     # PrioritySort (stable: creation order within a priority)
    pods.extend(queue)
    return nodes, pods, bound, P.default_profile()


def preemption_volume_case(n_nodes: int = 40, n_bound: int = 160, n_queue: int = 120, seed: int = 31):
    """preemption_case with claims: about half of the queued pods claim a
    zonal PV (VolumeZone), a local PV pinned to one or two hosts
    (VolumeBinding's node affinity), a plain PV or a ReadWriteOncePod claim
    that a running pod of higher priority than any preemptor holds
    (VolumeRestrictions).  In the default order VolumeRestrictions,
    VolumeBinding and VolumeZone follow NodeResourcesFit, so a node whose
    recorded rejection is Fit can still fail them in the dry run."""
    nodes, pods, bound, prof = preemption_case(n_nodes, n_bound, n_queue, seed)
    rng = np.random.Generator(np.random.PCG64(seed + 9191))
    st = m.Storage()
    done = {m.ANN_BIND_COMPLETED: "yes"}

    def claim(name, pv, modes=("ReadWriteOnce",)):
        st.pvs[pv.name] = pv
        pv.claim_ref = ("default", name)
        st.pvcs[("default", name)] = m.PersistentVolumeClaim(name, "default", pv.name, "", modes, dict(done))
    for z in range(4):
        claim(f"zonal-{z}", m.PersistentVolume(f"pv-zonal-{z}", labels={m.LABEL_ZONE: f"zone-{z}"}))
    for k in range(6):
        hosts = tuple(nodes[int(i)].name for i in rng.choice(len(nodes), size=1 + k % 2, replace=False))
        claim(f"local-{k}", m.PersistentVolume(f"pv-local-{k}", node_affinity=[
            m.NodeSelectorTerm(match_expressions=(m.Requirement(m.LABEL_HOSTNAME, m.IN, hosts),))]))
    claim("plain", m.PersistentVolume("pv-plain"))
    claim("rwop-0", m.PersistentVolume("pv-rwop-0"), ("ReadWriteOncePod",))
    shared = [f"zonal-{z}" for z in range(4)] + [f"local-{k}" for k in range(6)] + ["plain"]
    for p in pods:
        p.storage = st
    # the holder of rwop-0: a running pod no preemptor outranks
    holder = next(i for i, _ in bound if pods[i].node_name)
    pods[holder].priority = 5000
    pods[holder].volumes = [("v0", "persistentVolumeClaim", "rwop-0")]
    for p in pods[len(bound):]:
        if rng.random() < 0.5:
            p.volumes = [("v0", "persistentVolumeClaim", str(rng.choice(shared)))]
    # one queued claimant (the encoder refuses two queued users of one
    # ReadWriteOncePod claim)
    pods[len(bound)].volumes = [("v0", "persistentVolumeClaim", "rwop-0")]
    return nodes, pods, bound, prof


def preemption_topo_case(n_nodes: int = 40, n_bound: int = 160, n_queue: int = 120, seed: int = 21):
    """preemption_case with topology: running pods of six apps (a fifth with
    required hostname anti-affinity against another app), queued pods of
    higher priority with DoNotSchedule spread constraints (hostname or zone,
    on their own app), required anti-affinity (hostname) or required affinity
    (zone) — preemptors whose PodTopologySpread / InterPodAffinity verdicts
    change when victims leave the node.  Four zones, small nodes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes, pods, bound, prof = preemption_case(n_nodes=n_nodes, n_bound=n_bound, n_queue=n_queue, seed=seed)
    apps = [f"app-{k}" for k in range(6)]

    def sel(a):
        return m.LabelSelector(match_labels=(("app", a),))
    nb = len(bound)
    for p in pods[:nb]:
        p.labels = {"app": apps[int(rng.integers(len(apps)))]}
        if rng.random() < 0.20:
            other = apps[int(rng.integers(len(apps)))]
            p.pod_anti_affinity_required = [m.PodAffinityTerm(sel(other), m.LABEL_HOSTNAME)]
    for p in pods[nb:]:
        a = apps[int(rng.integers(len(apps)))]
        p.labels = {"app": a}
        u = rng.random()
        if u < 0.35:
            p.topology_spread_constraints = [m.TopologySpreadConstraint(1, m.LABEL_HOSTNAME, m.DO_NOT_SCHEDULE, sel(a))]
        elif u < 0.55:
            p.topology_spread_constraints = [m.TopologySpreadConstraint(int(rng.integers(1, 3)), m.LABEL_ZONE,
                                                                        m.DO_NOT_SCHEDULE, sel(a))]
        elif u < 0.75:
            other = apps[int(rng.integers(len(apps)))]
            p.pod_anti_affinity_required = [m.PodAffinityTerm(sel(other), m.LABEL_HOSTNAME)]
        elif u < 0.85:
            other = apps[int(rng.integers(len(apps)))]
            p.pod_affinity_required = [m.PodAffinityTerm(sel(other), m.LABEL_ZONE)]
    return nodes, pods, bound, prof


def preemption_ports_case(n_nodes: int = 40, n_bound: int = 160, n_queue: int = 120, seed: int = 31):
    """preemption_case with host ports: a third of the running pods and half
    of the queued pods hold a host port from a small set (8080/TCP on every
    IP, 9090/TCP, 53/UDP, 127.0.0.1:7000), so that queued pods meet NodePorts
    rejections a lower-priority victim's eviction resolves (DefaultPreemption
    with NodePorts re-run in the dry run)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes, pods, bound, prof = preemption_case(n_nodes=n_nodes, n_bound=n_bound, n_queue=n_queue, seed=seed)
    choices = [("", "", 8080), ("", "TCP", 9090), ("", "UDP", 53), ("127.0.0.1", "TCP", 7000)]
    nb = len(bound)
    used = {}   # node -> set of sanitised ports held by the running pods (no conflicts among them)
    for pi, ni in bound:
        if rng.random() < 0.33:
            hp = choices[int(rng.integers(len(choices)))]
            key = (m.sanitize_host_port(hp[0], hp[1]), hp[2])
            if key in used.setdefault(ni, set()):
                continue
            used[ni].add(key)
            pods[pi].containers[0].host_ports = (hp,)
    for p in pods[nb:]:
        if rng.random() < 0.5:
            p.containers[0].host_ports = (choices[int(rng.integers(len(choices)))],)
    return nodes, pods, bound, prof


def host_ports_case(n_nodes: int = 40, n_queue: int = 240, seed: int = 9, daemonset: bool = True):
    """NodePorts parity case.  Every node runs a DaemonSet-style pod already
    bound to it (hostPort 9100/TCP, as a node exporter; `daemonset`), ingested
    like any running pod.  The queue mixes: ingress pods on 80 + 443 (one per
    node at most), pods pinned to a host IP (127.0.0.1:8080 conflicts with a
    0.0.0.0:8080 pod and vice versa, 10.0.0.1:8080 does not conflict with
    127.0.0.1:8080), UDP/53 next to TCP/53 (different protocol: no
    conflict), a restartable init container (sidecar) holding 15000 (its
    ports count), a plain init container holding 15000 (its ports don't),
    a pod repeating its own port in two containers, DaemonSet-style pods
    for new ports with a matchFields node pin, and port-less pods.  Returns
    (nodes, pods, bound [(pod, node)], profile)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = [_node(i, rng, 4) for i in range(n_nodes)]
    pods, bound = [], []

    def pod(name, ports=(), init=None, req=None):
        c = m.Container(image="registry.k8s.io/pause:3.10", host_ports=tuple(ports),
                        requests=req if req is not None else {m.CPU: 100, m.MEMORY: 128 * MI})
        return m.Pod(name=name, containers=[c], init_containers=[init] if init else [])
    if daemonset:
        for i in range(n_nodes):
            p = pod(f"node-exporter-{i:04d}", [("", "", 9100)])
            p.node_name = nodes[i].name
            bound.append((len(pods), i))
            pods.append(p)
    kinds = ["ingress", "lo8080", "any8080", "ip8080", "dns-udp", "dns-tcp", "sidecar", "init", "dup",
             "exporter", "ds-new", "plain", "plain"]
    for j in range(n_queue):
        k = kinds[int(rng.integers(len(kinds)))]
        name = f"{k}-{j:05d}"
        if k == "ingress":
            p = pod(name, [("", "TCP", 80), ("", "TCP", 443)])
        elif k == "lo8080":
            p = pod(name, [("127.0.0.1", "TCP", 8080)])
        elif k == "any8080":
            p = pod(name, [("0.0.0.0", "", 8080)])
        elif k == "ip8080":
            p = pod(name, [("10.0.0.1", "TCP", 8080)])
        elif k == "dns-udp":
            p = pod(name, [("", "UDP", 53)])
        elif k == "dns-tcp":
            p = pod(name, [("", "TCP", 53), ("", "TCP", 0)])   # hostPort 0: not a host port
        elif k == "sidecar":
            p = pod(name, init=m.Container(image="envoy", restartable=True, host_ports=(("", "TCP", 15000),)))
        elif k == "init":
            p = pod(name, init=m.Container(image="busybox", host_ports=(("", "TCP", 15000),)))
        elif k == "dup":
            p = pod(name, [("", "TCP", 7000)])
            p.containers.append(m.Container(image="registry.k8s.io/pause:3.10", host_ports=(("", "TCP", 7000),)))
        elif k == "exporter":   # a second exporter asks for the DaemonSet's port
            p = pod(name, [("", "TCP", 9100)])
        elif k == "ds-new":     # DaemonSet controller: required matchFields metadata.name In [node]
            p = pod(name, [("", "TCP", 9200)])
            p.node_affinity_required = [m.NodeSelectorTerm(match_fields=(m.Requirement(
                m.OBJECT_NAME_FIELD, m.IN, (nodes[int(rng.integers(n_nodes))].name,)),))]
            p.tolerations.append(m.Toleration("", m.OP_EXISTS))
        else:
            p = pod(name)
        pods.append(p)
    return nodes, pods, bound, P.default_profile()
