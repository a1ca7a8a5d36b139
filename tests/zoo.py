"""Randomised small workloads that exercise the edge cases of every plugin:
hard and soft PodTopologySpread on zone / hostname / region, minDomains,
nodeAffinityPolicy / nodeTaintsPolicy, matchLabelKeys, system-default
spreading, InterPodAffinity required / preferred terms both ways, namespaces
and namespace selectors, node selectors with Gt/Lt/NotIn/DoesNotExist,
matchFields, nodes without labels, unschedulable nodes, NoExecute taints,
nodeName, init containers and sidecars, scalar resources, images; with
`ports`, host ports (NodePorts: bind-all vs specific host IPs, protocols,
sidecar ports) drawn from a separate stream so the other draws stay put."""
import numpy as np

from conftest import pkg

m = pkg("model")
P = pkg("profile")

GI = 1024 ** 3
MI = 1024 ** 2


def _sel(rng, apps):
    k = int(rng.integers(4))
    if k == 0:
        return m.LabelSelector(match_labels=(("app", f"a{int(rng.integers(apps))}"),))
    if k == 1:
        return m.LabelSelector(match_expressions=(m.Requirement("app", m.IN, tuple(
            f"a{int(x)}" for x in rng.integers(0, apps, size=2))),))
    if k == 2:
        return m.LabelSelector(match_labels=(("tier", "web"),),
                               match_expressions=(m.Requirement("app", m.EXISTS),))
    return m.LabelSelector(match_expressions=(m.Requirement("app", m.NOT_IN, (f"a{int(rng.integers(apps))}",)),))


PORTS = [("", "TCP", 80), ("", "TCP", 443), ("127.0.0.1", "TCP", 8080), ("0.0.0.0", "TCP", 8080),
         ("10.0.0.1", "", 8080), ("", "UDP", 53), ("", "TCP", 53), ("", "SCTP", 9000)]


def zoo(seed: int, n_nodes: int = 24, n_pods: int = 160, apps: int = 5, zones: int = 3, ports: bool = False):
    rng = np.random.Generator(np.random.PCG64(seed))
    prng = np.random.Generator(np.random.PCG64(seed + 7919))
    nodes = []
    for i in range(n_nodes):
        labels = {m.LABEL_HOSTNAME: f"n{i}", "rank": str(int(rng.integers(0, 20)))}
        if rng.random() > 0.1:
            labels[m.LABEL_ZONE] = f"z{int(rng.integers(zones))}"
        if rng.random() > 0.3:
            labels[m.LABEL_REGION] = f"r{int(rng.integers(2))}"
        if rng.random() < 0.05:
            labels = {}
        taints = []
        u = rng.random()
        if u < 0.15:
            taints.append(m.Taint("dedicated", "gpu", m.NO_SCHEDULE))
        elif u < 0.25:
            taints.append(m.Taint("flaky", "", m.NO_EXECUTE))
        if rng.random() < 0.3:
            taints.append(m.Taint("spot", "true", m.PREFER_NO_SCHEDULE))
        alloc = {m.CPU: int(rng.choice([2000, 4000, 8000])), m.MEMORY: int(rng.choice([4, 8, 16])) * GI,
                 m.EPHEMERAL: 20 * GI, m.PODS: int(rng.choice([8, 16, 110]))}
        if rng.random() < 0.3:
            alloc["example.com/fpga"] = int(rng.integers(1, 4))
        images = []
        if rng.random() < 0.6:
            images.append(m.ImageState(("registry/app:v1",), int(rng.integers(50, 900)) * MI))
        if rng.random() < 0.3:
            images.append(m.ImageState(("registry/db:v2", "registry/db@sha256:x"), 600 * MI))
        nodes.append(m.Node(name=f"n{i}", labels=labels, taints=taints, allocatable=alloc,
                            unschedulable=bool(rng.random() < 0.05), images=images))
    pods = []
    for j in range(n_pods):
        ns = "default" if rng.random() < 0.8 else "other"
        app = f"a{int(rng.integers(apps))}"
        labels = {"app": app}
        if rng.random() < 0.5:
            labels["tier"] = "web"
        req = {}
        if rng.random() > 0.1:
            req = {m.CPU: int(rng.choice([100, 250, 500, 1000])), m.MEMORY: int(rng.choice([256, 512, 1024])) * MI}
        if rng.random() < 0.1:
            req["example.com/fpga"] = 1
        if rng.random() < 0.1:
            req[m.EPHEMERAL] = GI
        conts = [m.Container(image=str(rng.choice(["registry/app:v1", "registry/app", "registry/db:v2"])),
                             requests=req)]
        inits = []
        if rng.random() < 0.1:
            inits.append(m.Container(image="busybox", requests={m.CPU: 1500}))
        if rng.random() < 0.05:
            inits.append(m.Container(image="registry/db:v2", requests={m.MEMORY: 64 * MI}, restartable=True))
        p = m.Pod(name=f"p{j}", namespace=ns, labels=labels, containers=conts, init_containers=inits)
        if rng.random() < 0.15:
            p.tolerations.append(m.Toleration("dedicated", m.OP_EQUAL, "gpu", m.NO_SCHEDULE))
        if rng.random() < 0.1:
            p.tolerations.append(m.Toleration("", m.OP_EXISTS))
        if rng.random() < 0.1:
            p.tolerations.append(m.Toleration("spot", m.OP_EXISTS, "", m.PREFER_NO_SCHEDULE))
        if rng.random() < 0.05:
            p.tolerations.append(m.Toleration(m.TAINT_NODE_UNSCHEDULABLE, m.OP_EXISTS, "", m.NO_SCHEDULE))
        if rng.random() < 0.1:
            p.node_selector = {m.LABEL_REGION: f"r{int(rng.integers(2))}"}
        if rng.random() < 0.15:
            op = rng.choice([m.GT, m.LT, m.NOT_IN, m.DOES_NOT_EXIST, m.IN])
            if op in (m.GT, m.LT):
                r = m.Requirement("rank", str(op), (str(int(rng.integers(0, 20))),))
            elif op == m.DOES_NOT_EXIST:
                r = m.Requirement(m.LABEL_REGION, m.DOES_NOT_EXIST)
            else:
                r = m.Requirement(m.LABEL_ZONE, str(op), (f"z{int(rng.integers(zones))}",))
            terms = [m.NodeSelectorTerm(match_expressions=(r,))]
            if rng.random() < 0.3:
                terms.append(m.NodeSelectorTerm(match_fields=(m.Requirement(
                    m.OBJECT_NAME_FIELD, m.IN, (f"n{int(rng.integers(n_nodes))}",)),)))
            p.node_affinity_required = terms
        if rng.random() < 0.15:
            p.node_affinity_preferred = [m.PreferredSchedulingTerm(int(rng.integers(1, 100)), m.NodeSelectorTerm(
                match_expressions=(m.Requirement(m.LABEL_ZONE, m.IN, (f"z{int(rng.integers(zones))}",)),)))]
        if rng.random() < 0.03:
            p.node_name = f"n{int(rng.integers(n_nodes))}"
        # PodTopologySpread
        u = rng.random()
        if u < 0.35:
            cons = []
            for _ in range(int(rng.integers(1, 3))):
                key = str(rng.choice([m.LABEL_ZONE, m.LABEL_HOSTNAME, m.LABEL_REGION]))
                when = m.DO_NOT_SCHEDULE if rng.random() < 0.5 else m.SCHEDULE_ANYWAY
                cons.append(m.TopologySpreadConstraint(
                    int(rng.integers(1, 4)), key, when,
                    m.LabelSelector(match_labels=(("app", app),)) if rng.random() < 0.8 else _sel(rng, apps),
                    min_domains=int(rng.integers(1, 5)) if (when == m.DO_NOT_SCHEDULE and rng.random() < 0.3) else None,
                    node_affinity_policy=m.POLICY_IGNORE if rng.random() < 0.2 else None,
                    node_taints_policy=m.POLICY_HONOR if rng.random() < 0.3 else None,
                    match_label_keys=("tier",) if rng.random() < 0.2 else ()))
            p.topology_spread_constraints = cons
        elif u < 0.45:
            p.default_spread_selector = m.LabelSelector(match_labels=(("app", app),))
        # InterPodAffinity
        if rng.random() < 0.15:
            p.pod_affinity_required = [m.PodAffinityTerm(_sel(rng, apps), str(rng.choice(
                [m.LABEL_ZONE, m.LABEL_HOSTNAME])))]
        if rng.random() < 0.15:
            t = m.PodAffinityTerm(m.LabelSelector(match_labels=(("app", app),)), m.LABEL_HOSTNAME,
                                  namespaces=("default", "other") if rng.random() < 0.3 else ())
            p.pod_anti_affinity_required = [t]
        if rng.random() < 0.2:
            p.pod_affinity_preferred = [m.WeightedPodAffinityTerm(int(rng.integers(1, 100)), m.PodAffinityTerm(
                _sel(rng, apps), m.LABEL_ZONE,
                namespace_selector=m.LabelSelector() if rng.random() < 0.3 else None))]
        if rng.random() < 0.2:
            p.pod_anti_affinity_preferred = [m.WeightedPodAffinityTerm(int(rng.integers(1, 100)), m.PodAffinityTerm(
                m.LabelSelector(match_labels=(("app", app),)), str(rng.choice([m.LABEL_ZONE, m.LABEL_HOSTNAME]))))]
        if ports and prng.random() < 0.3:
            hp = tuple(PORTS[int(k)] for k in prng.choice(len(PORTS), size=int(prng.integers(1, 3)), replace=False))
            if prng.random() < 0.2:
                p.init_containers.append(m.Container(image="envoy", restartable=bool(prng.random() < 0.7),
                                                     host_ports=hp))
            else:
                p.containers[0].host_ports = hp
        pods.append(p)
    prof = P.default_profile()
    if seed % 3 == 1:
        prof.fit_strategy = P.MOST_ALLOCATED
        prof.fit_resources = [(m.CPU, 2), (m.MEMORY, 1), ("example.com/fpga", 3)]
        prof.ba_resources = [(m.CPU, 1), (m.MEMORY, 1), (m.EPHEMERAL, 1)]
    if seed % 4 == 2:
        prof.hard_pod_affinity_weight = 5
    return nodes, pods, prof


# shapes of NodeResourcesFit RequestedToCapacityRatio (utilization, score 0..10):
# bin packing, spreading, and one starting above 0 % and ending below 100 %
RTCR_SHAPES = [[(0, 0), (100, 10)], [(0, 10), (40, 6), (100, 0)], [(20, 3), (60, 9), (90, 2)]]


def zoo_args(seed: int, kind: str, **kw):
    """zoo() under a profile with the plugin args the evaluator models beyond
    the defaults: "rtcr" (NodeResourcesFit RequestedToCapacityRatio, a shape
    per seed) or "pts-list" (PodTopologySpread defaultingType List with
    defaultConstraints, hard and soft, applied to the pods that have owners
    but no constraints of their own)."""
    nodes, pods, prof = zoo(seed, **kw)
    if kind == "rtcr":
        prof.fit_strategy = P.REQUESTED_TO_CAPACITY_RATIO
        prof.fit_shape = list(RTCR_SHAPES[seed % len(RTCR_SHAPES)])
    elif kind == "pts-list":
        prof.pts_system_defaulted = False
        prof.pts_default_constraints = [
            m.TopologySpreadConstraint(1 + seed % 2, m.LABEL_ZONE, m.DO_NOT_SCHEDULE, None),
            m.TopologySpreadConstraint(2, m.LABEL_HOSTNAME, m.SCHEDULE_ANYWAY, None,
                                       node_taints_policy=m.POLICY_HONOR if seed % 2 else None),
        ]
    else:
        raise ValueError(kind)
    return nodes, pods, prof


def zoo_volumes(seed: int, n_nodes: int = 30, n_pods: int = 90, bound: bool = False):
    """Pods with persistentVolumeClaim volumes over a cluster with zones and
    regions (GA and beta labels), exercising VolumeRestrictions,
    NodeVolumeLimits, VolumeBinding and VolumeZone: local PVs pinned by
    hostname (VolumeBinding's PreFilterResult), zonal PVs (single and
    "__"-joined multi-zone labels, beta keys matched against GA node labels),
    PVs with zone node affinity, claims bound to missing PVs, claims without
    bind-completed (unbound immediate), WaitForFirstConsumer claims against
    classes with allowedTopologies / no provisioner / a selected node, missing
    claims and ReadWriteOncePod claims.  bound=True also returns running pods
    [(pod index, node index)] that hold some ReadWriteOncePod claims."""
    rng = np.random.Generator(np.random.PCG64(seed + 4242))
    nodes, pods, prof = zoo(seed, n_nodes=n_nodes, n_pods=n_pods)
    zones = [f"z{k}" for k in range(3)]
    for i, n in enumerate(nodes):
        if not n.labels:
            continue
        z = zones[i % 3]
        u = rng.random()
        if u < 0.5:
            n.labels[m.LABEL_ZONE] = z
            n.labels["topology.kubernetes.io/region"] = "r0"
        elif u < 0.7:
            n.labels[m.LABEL_BETA_ZONE] = z
        elif u < 0.8:
            n.labels.pop(m.LABEL_ZONE, None)
            n.labels.pop(m.LABEL_REGION, None)
    st = m.Storage()
    st.classes["fast"] = m.StorageClass("fast", "csi.example.com", m.BINDING_WAIT_FOR_FIRST_CONSUMER,
                                        (((m.LABEL_ZONE, ("z0", "z1")),), (("topology.kubernetes.io/region", ("r9",)),)))
    st.classes["any"] = m.StorageClass("any", "csi.example.com", m.BINDING_WAIT_FOR_FIRST_CONSUMER)
    st.classes["local"] = m.StorageClass("local", m.NOT_SUPPORTED_PROVISIONER, m.BINDING_WAIT_FOR_FIRST_CONSUMER)
    st.classes["imm"] = m.StorageClass("imm", "csi.example.com", m.BINDING_IMMEDIATE)
    done = {m.ANN_BIND_COMPLETED: "yes"}

    nss = sorted({p.namespace for p in pods} | {"default"})

    def bound_claim(name, pv, modes=("ReadWriteOnce",)):
        st.pvs[pv.name] = pv
        pv.claim_ref = ("default", name)
        for ns in nss:   # the same claim name in every namespace (all bound to the one PV)
            st.pvcs[(ns, name)] = m.PersistentVolumeClaim(name, ns, pv.name, pv.storage_class, modes, dict(done))

    hosts = [n.name for n in nodes if n.labels.get(m.LABEL_HOSTNAME)]
    for k in range(6):   # local PVs pinned to one or two hosts
        names = tuple(rng.choice(hosts, size=1 + k % 2, replace=False))
        bound_claim(f"local-{k}", m.PersistentVolume(f"pv-local-{k}", storage_class="x", node_affinity=[
            m.NodeSelectorTerm(match_expressions=(m.Requirement(m.LABEL_HOSTNAME, m.IN, names),))]))
    for k, z in enumerate(["z0", "z1", "z0__z2", "z2"]):   # zonal PVs (labels)
        key = m.LABEL_BETA_ZONE if k % 2 else m.LABEL_ZONE
        bound_claim(f"zonal-{k}", m.PersistentVolume(f"pv-zonal-{k}", labels={key: z}))
    bound_claim("zonal-region", m.PersistentVolume("pv-zonal-region", labels={m.LABEL_BETA_REGION: "r0"}))
    bound_claim("aff-zone", m.PersistentVolume("pv-aff-zone", node_affinity=[
        m.NodeSelectorTerm(match_expressions=(m.Requirement(m.LABEL_ZONE, m.IN, ("z1", "z2")),)),
        m.NodeSelectorTerm(match_fields=(m.Requirement(m.OBJECT_NAME_FIELD, m.IN, ("nowhere",)),),
                           match_expressions=(m.Requirement("rank", m.GT, ("15",)),))]))
    bound_claim("plain", m.PersistentVolume("pv-plain"))
    st.pvcs[("default", "ghost")] = m.PersistentVolumeClaim("ghost", "default", "pv-missing", "", ("ReadWriteOnce",),
                                                            dict(done))
    st.pvcs[("default", "prebound")] = m.PersistentVolumeClaim("prebound", "default", "pv-plain", "",
                                                               ("ReadWriteOnce",))
    st.pvcs[("default", "immediate")] = m.PersistentVolumeClaim("immediate", "default", "", "imm")
    for k in range(3):
        bound_claim(f"rwop-{k}", m.PersistentVolume(f"pv-rwop-{k}"), ("ReadWriteOncePod",))
    shared = ["local-0", "local-1", "local-2", "local-3", "local-4", "local-5", "zonal-0", "zonal-1", "zonal-2",
              "zonal-3", "zonal-region", "aff-zone", "plain", "ghost", "prebound", "immediate", "missing"]
    for i, p in enumerate(pods):
        p.storage = st
        u = rng.random()
        if u < 0.35:
            continue
        if u < 0.75:
            cs = list(rng.choice(shared, size=1 + int(rng.random() < 0.3), replace=False))
        else:   # a claim of its own: WaitForFirstConsumer (maybe with a selected node)
            cls = ["fast", "any", "local"][int(rng.integers(3))]
            ann = {}
            if rng.random() < 0.2:
                ann[m.ANN_SELECTED_NODE] = nodes[int(rng.integers(len(nodes)))].name
            name = f"own-{i}"
            st.pvcs[(p.namespace, name)] = m.PersistentVolumeClaim(name, p.namespace, "", cls, ("ReadWriteOnce",),
                                                                   ann)
            cs = [name]
            if rng.random() < 0.3:
                cs.append(str(rng.choice(["zonal-0", "local-2", "plain"])))
        p.volumes = [(f"v{k}", "persistentVolumeClaim", c) for k, c in enumerate(cs)]
    if not bound:
        return nodes, pods, prof
    # two running pods hold rwop-0 / rwop-1; queued pods claim rwop-0..2
    run = []
    for k in range(2):
        q = m.Pod(name=f"holder-{k}", containers=[m.Container(requests={m.CPU: 100})], storage=st,
                  volumes=[("v0", "persistentVolumeClaim", f"rwop-{k}")])
        pods.insert(k, q)
        run.append((k, k))
    for j, i in enumerate(range(2, len(pods), 9)):
        if j < 3:
            pods[i].volumes = [("v0", "persistentVolumeClaim", f"rwop-{j}")]
    return nodes, pods, prof, run
