"""Scheduler profile: which plugins run, in which order, with which weights/args.

Mirrors what the debuggable scheduler derives from a KubeSchedulerConfiguration:
- the MultiPoint plugin order after `ConvertForSimulator`
  (`simulator/scheduler/plugin/plugins.go:174-197`; the converted default
  profile is pinned at `simulator/scheduler/scheduler_test.go:519-541`),
- the score-weight map of `getScorePluginWeight` (`plugins.go:289-304`: weight
  0 maps to 1, key is the plugin name without the `Wrapped` suffix),
- the default plugin args pinned at `plugins_test.go:876-1000`
  (LeastAllocated cpu=1/memory=1, BalancedAllocation cpu=1/memory=1,
  hardPodAffinityWeight=1, PodTopologySpread defaultingType System),
- per-extension-point plugin sets (`Profile.points`): ConvertForSimulator keeps
  them as written (`plugins.go:177-186`) beside the in-tree MultiPoint set
  (`plugins.go:187-194`); the framework then expands MultiPoint into each
  point [upstream v1.32 frameworkImpl.expandMultiPointPlugins, not vendored —
  TO VERIFY, DESIGN.md §9]: the point's own plugins that MultiPoint also
  lists first (in the point's order), then the remaining MultiPoint plugins
  that implement the point and are not disabled there, then the point's other
  plugins.  Score weights differ by consumer: the framework's selection takes
  a point's own Score weight before the MultiPoint one [upstream
  getScoreWeights, TO VERIFY], while the simulator's store map appends
  MultiPoint after Score.Enabled, so the MultiPoint weight wins there
  (`plugins.go:289-304`) and the finalscore annotations use it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import model as m

PLUGIN_SUFFIX = "Wrapped"  # wrappedplugin.go:242-248

# Stable plugin ids shared with include/ksched.h (KSG_PL_*).
NODE_UNSCHEDULABLE = 0
NODE_NAME = 1
TAINT_TOLERATION = 2
NODE_AFFINITY = 3
NODE_PORTS = 4
NODE_RESOURCES_FIT = 5
VOLUME_RESTRICTIONS = 6
NODE_VOLUME_LIMITS = 7
VOLUME_BINDING = 8
VOLUME_ZONE = 9
POD_TOPOLOGY_SPREAD = 10
INTER_POD_AFFINITY = 11
BALANCED_ALLOCATION = 12
IMAGE_LOCALITY = 13
N_PLUGINS = 14

PLUGIN_NAMES = [
    "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
    "NodeResourcesFit", "VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding",
    "VolumeZone", "PodTopologySpread", "InterPodAffinity",
    "NodeResourcesBalancedAllocation", "ImageLocality",
]
PLUGIN_ID = {n: i for i, n in enumerate(PLUGIN_NAMES)}

# Plugins of the default profile that take part in neither Filter nor Score.
NON_EVAL_PLUGINS = ("SchedulingGates", "PrioritySort", "DefaultPreemption", "DefaultBinder")

# Extension points each in-tree plugin implements in kube-scheduler v1.32
# [upstream, TO VERIFY — source not in container, SURVEY.md §8(c)].
# (prefilter, filter, prescore, score, normalize)
EXT = {
    NODE_UNSCHEDULABLE: (False, True, False, False, False),
    NODE_NAME: (False, True, False, False, False),
    TAINT_TOLERATION: (False, True, True, True, True),
    NODE_AFFINITY: (True, True, True, True, True),
    NODE_PORTS: (True, True, False, False, False),
    NODE_RESOURCES_FIT: (True, True, True, True, False),
    VOLUME_RESTRICTIONS: (True, True, False, False, False),
    NODE_VOLUME_LIMITS: (True, True, False, False, False),
    VOLUME_BINDING: (True, True, True, True, False),
    VOLUME_ZONE: (True, True, False, False, False),
    POD_TOPOLOGY_SPREAD: (True, True, True, True, True),
    INTER_POD_AFFINITY: (True, True, True, True, True),
    BALANCED_ALLOCATION: (False, False, True, True, False),
    IMAGE_LOCALITY: (False, False, False, True, False),
}

LEAST_ALLOCATED = 0
MOST_ALLOCATED = 1
REQUESTED_TO_CAPACITY_RATIO = 2
STRATEGY_NAMES = {"LeastAllocated": LEAST_ALLOCATED, "MostAllocated": MOST_ALLOCATED,
                  "RequestedToCapacityRatio": REQUESTED_TO_CAPACITY_RATIO}
MAX_SHAPE = 16            # KSG_MAX_SHAPE: shape points the evaluator carries
MAX_CUSTOM_PRIORITY_SCORE = 10   # a shape point's score range (config.MaxCustomPriorityScore)

DEFAULT_MULTIPOINT: List[Tuple[str, int]] = [
    ("SchedulingGates", 0), ("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0),
    ("TaintToleration", 3), ("NodeAffinity", 2), ("NodePorts", 0), ("NodeResourcesFit", 1),
    ("VolumeRestrictions", 0), ("NodeVolumeLimits", 0), ("VolumeBinding", 0), ("VolumeZone", 0),
    ("PodTopologySpread", 2), ("InterPodAffinity", 2), ("DefaultPreemption", 0),
    ("NodeResourcesBalancedAllocation", 1), ("ImageLocality", 1), ("DefaultBinder", 0),
]


@dataclass
class Profile:
    """One KubeSchedulerProfile as the debuggable scheduler runs it."""
    plugins: List[Tuple[str, int]] = field(default_factory=lambda: list(DEFAULT_MULTIPOINT))
    fit_strategy: int = LEAST_ALLOCATED
    fit_resources: List[Tuple[str, int]] = field(default_factory=lambda: [(m.CPU, 1), (m.MEMORY, 1)])
    ba_resources: List[Tuple[str, int]] = field(default_factory=lambda: [(m.CPU, 1), (m.MEMORY, 1)])
    fit_ignored_resources: Tuple[str, ...] = ()
    fit_ignored_resource_groups: Tuple[str, ...] = ()
    hard_pod_affinity_weight: int = 1
    ignore_preferred_terms_of_existing_pods: bool = False
    # NodeResourcesFitArgs.scoringStrategy.requestedToCapacityRatio.shape:
    # (utilization 0..100 increasing, score 0..10) points as written
    fit_shape: List[Tuple[int, int]] = field(default_factory=list)
    # PodTopologySpreadArgs.defaultingType == System (no explicit defaultConstraints)
    pts_system_defaulted: bool = True
    # PodTopologySpreadArgs.defaultConstraints (defaultingType List): the
    # constraints a pod without its own gets, with the selector of its owning
    # services / controllers (buildDefaultConstraints); label_selector unset
    pts_default_constraints: List[m.TopologySpreadConstraint] = field(default_factory=list)
    # BalancedAllocation PreScore Skip for best-effort pods [upstream; believed
    # to land after v1.32 — TO VERIFY, SURVEY.md Appendix A.2]
    ba_skip_best_effort: bool = False
    # DefaultPreemptionArgs (v1 defaults): candidate count =
    # max(potential nodes * pct / 100, abs), at most the potential nodes
    preemption_min_candidate_pct: int = 10
    preemption_min_candidate_abs: int = 100
    # per-extension-point sets: point ("preFilter", "filter", "preScore",
    # "score") -> (enabled [(name, weight)], disabled names)
    points: Dict[str, Tuple[List[Tuple[str, int]], Tuple[str, ...]]] = field(default_factory=dict)

    def validate_args(self) -> None:
        """The plugin-args rules the scheduler's config validation applies to
        the args modelled here [upstream v1.32 apis/config/validation/
        validation_pluginargs.go: ValidateNodeResourcesFitArgs' shape rules,
        ValidatePodTopologySpreadArgs]; ValueError on a configuration the
        reference's scheduler would refuse to start with."""
        if self.fit_strategy == REQUESTED_TO_CAPACITY_RATIO:
            if not self.fit_shape:
                raise ValueError("requestedToCapacityRatio.shape: at least one point must be specified")
            if len(self.fit_shape) > MAX_SHAPE:
                raise NotImplementedError(f"requestedToCapacityRatio.shape: more than {MAX_SHAPE} points")
            for i, (u, sc) in enumerate(self.fit_shape):
                if not 0 <= u <= 100:
                    raise ValueError(f"shape[{i}].utilization {u} not in [0, 100]")
                if i and u <= self.fit_shape[i - 1][0]:
                    raise ValueError("shape utilization values must be sorted in increasing order")
                if not 0 <= sc <= MAX_CUSTOM_PRIORITY_SCORE:
                    raise ValueError(f"shape[{i}].score {sc} not in [0, {MAX_CUSTOM_PRIORITY_SCORE}]")
        if self.pts_system_defaulted and self.pts_default_constraints:
            raise ValueError("defaultConstraints must be empty when defaultingType is System")
        seen = set()
        for i, c in enumerate(self.pts_default_constraints):
            if c.max_skew <= 0:
                raise ValueError(f"defaultConstraints[{i}].maxSkew must be greater than zero")
            if not c.topology_key:
                raise ValueError(f"defaultConstraints[{i}].topologyKey can not be empty")
            if c.when_unsatisfiable not in (m.DO_NOT_SCHEDULE, m.SCHEDULE_ANYWAY):
                raise ValueError(f"defaultConstraints[{i}].whenUnsatisfiable {c.when_unsatisfiable!r}")
            if (c.topology_key, c.when_unsatisfiable) in seen:
                raise ValueError(f"defaultConstraints[{i}]: duplicate (topologyKey, whenUnsatisfiable)")
            seen.add((c.topology_key, c.when_unsatisfiable))
            if c.label_selector is not None:
                raise ValueError(f"defaultConstraints[{i}]: constraint must not define a selector")

    # -- derived views ---------------------------------------------------
    def enabled_ids(self) -> List[int]:
        """Filter/score-relevant plugin ids in MultiPoint order."""
        out = []
        for name, _ in self.plugins:
            name = name[:-len(PLUGIN_SUFFIX)] if name.endswith(PLUGIN_SUFFIX) else name
            if name in PLUGIN_ID:
                out.append(PLUGIN_ID[name])
            elif name not in NON_EVAL_PLUGINS:
                raise ValueError(f"plugin {name!r} is not an in-tree Filter/Score plugin")
        return out

    def _expand(self, point: str, ext: int) -> List[int]:
        """The framework's plugin list of one extension point (module docstring)."""
        multi = [p for p in self.enabled_ids() if EXT[p][ext]]
        if point not in self.points:
            return multi
        enabled, disabled = self.points[point]
        own = [_plain(n) for n, _ in enabled]
        for n in own:   # updatePluginList: the plugin must exist and implement the point
            if n not in PLUGIN_ID:
                raise ValueError(f"plugin {n!r} in {point!r} is not an in-tree Filter/Score plugin")
            if not EXT[PLUGIN_ID[n]][ext]:
                raise ValueError(f"plugin {n!r} does not extend {point!r}")
        own_ids = [PLUGIN_ID[n] for n in own]
        if len(set(own_ids)) != len(own_ids):
            raise ValueError(f"plugin listed twice in {point!r}")
        if "*" in disabled:
            return own_ids
        off = {PLUGIN_ID[_plain(n)] for n in disabled if _plain(n) in PLUGIN_ID}
        override = [p for p in own_ids if p in multi]
        rest_multi = [p for p in multi if p not in off and p not in own_ids]
        return override + rest_multi + [p for p in own_ids if p not in multi]

    def filter_order(self) -> List[int]:
        return self._expand("filter", 1)

    def prefilter_order(self) -> List[int]:
        return self._expand("preFilter", 0)

    def prescore_order(self) -> List[int]:
        return self._expand("preScore", 2)

    def score_order(self) -> List[int]:
        return self._expand("score", 3)

    def weights(self) -> Dict[str, int]:
        """getScorePluginWeight (plugins.go:289-304), the store's map:
        Score.Enabled, then every enabled MultiPoint plugin (a later entry
        replaces an earlier one); weight 0 is replaced by 1."""
        out = {}
        for name, w in list(self.points.get("score", ([], ()))[0]) + list(self.plugins):
            out[_plain(name)] = w if w != 0 else 1
        return out

    def selection_weights(self) -> Dict[str, int]:
        """The framework's Score weights (selection): a point's own Score
        weight first, then MultiPoint's (the first entry wins); 0 -> 1."""
        out: Dict[str, int] = {}
        for name, w in list(self.points.get("score", ([], ()))[0]) + list(self.plugins):
            out.setdefault(_plain(name), w if w != 0 else 1)
        return out

    def weight_of(self, pid: int) -> int:
        return self.weights().get(PLUGIN_NAMES[pid], 0)

    def simulator_plugin_names(self) -> List[str]:
        """Names after ConvertForSimulator (plugins.go:174-197)."""
        return [n if n.endswith(PLUGIN_SUFFIX) else n + PLUGIN_SUFFIX for n, _ in self.plugins]


def _plain(name: str) -> str:
    return name[:-len(PLUGIN_SUFFIX)] if name.endswith(PLUGIN_SUFFIX) else name


def default_profile() -> Profile:
    return Profile()


def config2_profile(strategy: int = LEAST_ALLOCATED, weights: Optional[Dict[str, int]] = None) -> Profile:
    """BASELINE.json configs[1]: NodeResourcesFit + BalancedAllocation +
    TaintToleration + NodeAffinity (plus the cheap always-on filters)."""
    w = {"TaintToleration": 3, "NodeAffinity": 2, "NodeResourcesFit": 1,
         "NodeResourcesBalancedAllocation": 1}
    if weights:
        w.update(weights)
    plugins = [("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0),
               ("TaintToleration", w["TaintToleration"]), ("NodeAffinity", w["NodeAffinity"]),
               ("NodeResourcesFit", w["NodeResourcesFit"]),
               ("NodeResourcesBalancedAllocation", w["NodeResourcesBalancedAllocation"]),
               ("DefaultBinder", 0)]
    return Profile(plugins=plugins, fit_strategy=strategy)


def config3_profile() -> Profile:
    """BASELINE.json configs[2]: config 2 plus PodTopologySpread and InterPodAffinity."""
    plugins = [("PrioritySort", 0), ("NodeUnschedulable", 0), ("NodeName", 0),
               ("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
               ("PodTopologySpread", 2), ("InterPodAffinity", 2),
               ("NodeResourcesBalancedAllocation", 1), ("DefaultBinder", 0)]
    return Profile(plugins=plugins)
