// Profile construction from the scheduler configuration and the plugin
// factories' decoded args.  Source only: no Go toolchain in this image
// (DESIGN.md §1).
package ksched

import (
	"fmt"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/runtime"
	configv1 "k8s.io/kube-scheduler/config/v1"
	"k8s.io/kubernetes/pkg/scheduler/apis/config"
)

// ProfileFromConfig mirrors profile 0 of the converted configuration the
// debuggable scheduler runs (ConvertForSimulator, plugins.go:174-197):
// MultiPoint.Enabled in order and the PreFilter / Filter / PreScore / Score
// sets as written.  Plugin args start at the v1 defaults
// (plugins_test.go:876-1000) and are overwritten by ApplyPluginArgs when the
// framework hands each factory its decoded args.
func ProfileFromConfig(p *configv1.KubeSchedulerProfile) *ProfileArgs {
	out := &ProfileArgs{
		FitStrategy:           "LeastAllocated",
		FitResources:          map[string]int64{"cpu": 1, "memory": 1},
		FitResourceOrder:      []string{"cpu", "memory"},
		BAResources:           map[string]int64{"cpu": 1, "memory": 1},
		BAResourceOrder:       []string{"cpu", "memory"},
		HardPodAffinityWeight: 1,
		PTSSystemDefaulted:    true,
	}
	if p.Plugins == nil {
		return out
	}
	conv := func(ps configv1.PluginSet) PluginSet {
		var s PluginSet
		for _, e := range ps.Enabled {
			w := int32(0)
			if e.Weight != nil {
				w = *e.Weight
			}
			s.Enabled = append(s.Enabled, Plugin{Name: e.Name, Weight: w})
		}
		for _, d := range ps.Disabled {
			s.Disabled = append(s.Disabled, d.Name)
		}
		return s
	}
	out.Plugins = conv(p.Plugins.MultiPoint).Enabled
	out.Points[PointPreFilter] = conv(p.Plugins.PreFilter)
	out.Points[PointFilter] = conv(p.Plugins.Filter)
	out.Points[PointPreScore] = conv(p.Plugins.PreScore)
	out.Points[PointScore] = conv(p.Plugins.Score)
	return out
}

// ApplyPluginArgs records the args the framework decoded for plugin `name`
// (the runtime.Object its factory receives: internal config types of
// k8s.io/kubernetes/pkg/scheduler/apis/config).  Settings the evaluator does
// not model are refused instead of ignored.
func (p *ProfileArgs) ApplyPluginArgs(name string, obj runtime.Object) error {
	if obj == nil {
		return nil
	}
	switch a := obj.(type) {
	case *config.NodeResourcesFitArgs:
		if a.ScoringStrategy != nil {
			switch a.ScoringStrategy.Type {
			case config.LeastAllocated, config.MostAllocated:
				p.FitStrategy = string(a.ScoringStrategy.Type)
				p.FitShape = nil
			case config.RequestedToCapacityRatio:
				p.FitStrategy = string(a.ScoringStrategy.Type)
				p.FitShape = nil
				if r := a.ScoringStrategy.RequestedToCapacityRatio; r != nil {
					for _, pt := range r.Shape {
						p.FitShape = append(p.FitShape, [2]int32{pt.Utilization, pt.Score})
					}
				}
			default:
				return fmt.Errorf("ksched: NodeResourcesFit scoring strategy %q is not modelled", a.ScoringStrategy.Type)
			}
			if len(a.ScoringStrategy.Resources) > 0 {
				p.FitResources, p.FitResourceOrder = map[string]int64{}, nil
				for _, r := range a.ScoringStrategy.Resources {
					p.FitResources[r.Name] = r.Weight
					p.FitResourceOrder = append(p.FitResourceOrder, r.Name)
				}
			}
		}
		p.FitIgnoredResources = append([]string(nil), a.IgnoredResources...)
		p.FitIgnoredGroups = append([]string(nil), a.IgnoredResourceGroups...)
	case *config.NodeResourcesBalancedAllocationArgs:
		if len(a.Resources) > 0 {
			p.BAResources, p.BAResourceOrder = map[string]int64{}, nil
			for _, r := range a.Resources {
				p.BAResources[r.Name] = r.Weight
				p.BAResourceOrder = append(p.BAResourceOrder, r.Name)
			}
		}
	case *config.InterPodAffinityArgs:
		p.HardPodAffinityWeight = a.HardPodAffinityWeight
		p.IgnorePreferredTermsOfExistingPods = a.IgnorePreferredTermsOfExistingPods
	case *config.PodTopologySpreadArgs:
		// the snapshot validates defaultConstraints as the scheduler does
		// (ksg_snapshot_new refuses a System profile that lists any)
		p.PTSSystemDefaulted = a.DefaultingType == config.SystemDefaulting
		p.PTSDefaultConstraints = append([]v1.TopologySpreadConstraint(nil), a.DefaultConstraints...)
	case *config.NodeAffinityArgs:
		if a.AddedAffinity != nil {
			return fmt.Errorf("ksched: NodeAffinity addedAffinity is not modelled")
		}
	default:
		// plugins without modelled args (TaintToleration, ImageLocality, ...)
	}
	return nil
}
