// Package gpuplugins exposes the MI355X evaluator as in-tree-named Scheduling
// Framework plugins, so the simulator's wrappedPlugin and resultstore.Store
// stay unchanged (SURVEY.md §8(b)).  Source only (no Go toolchain here).
//
// Wiring: overlay these factories onto the in-tree registry returned at
// simulator/scheduler/config/plugin.go:49-51 (plugins.go:50 looks in-tree up
// first), or add an option next to debuggablescheduler.WithPlugin
// (simulator/pkg/debuggablescheduler/command.go:64-68).  Name() returns the
// in-tree name, so Store keys (wrappedplugin.go:406,438,542) and
// getScorePluginWeight (plugins.go:295) see the same names as today.
package gpuplugins

import (
	"context"
	"fmt"
	"sync"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/kubernetes/pkg/scheduler/framework"

	"example.invalid/ksched-mi355x/shim/go/ksched"
)

const stateKey framework.StateKey = "ksched/eval"

// podState is the per-pod SoA result, computed once at PreFilter time.
type podState struct {
	ev    *ksched.PodEval
	index map[string]int // node name -> column
}

func (s *podState) Clone() framework.StateData { return s }

// Evaluator owns the device context and the host-side encoder (the Go
// equivalent of encoder.py: NodeInfo/PodInfo -> SoA columns + pod programs).
type Evaluator struct {
	mu    sync.Mutex
	ctx   *ksched.Ctx
	enc   Encoder
	names []string
}

// Encoder is the snapshot/pod encoder (encoder.py restated in Go).
type Encoder interface {
	// SyncNodes re-encodes the snapshot when it changed; returns node names in column order.
	SyncNodes(ctx *ksched.Ctx, nodes []*framework.NodeInfo) ([]string, error)
	// LoadPod encodes one pod as a single-pod workload (index 0).
	LoadPod(ctx *ksched.Ctx, pod *v1.Pod) error
	// Message rebuilds the upstream status message from a filter status word.
	Message(plugin int, word uint32, node string) (framework.Code, string)
}

func (e *Evaluator) evalPod(ctx context.Context, cs *framework.CycleState, pod *v1.Pod,
	nodes []*framework.NodeInfo) (*podState, error) {
	if d, err := cs.Read(stateKey); err == nil {
		return d.(*podState), nil
	}
	e.mu.Lock()
	defer e.mu.Unlock()
	names, err := e.enc.SyncNodes(e.ctx, nodes)
	if err != nil {
		return nil, err
	}
	if err := e.enc.LoadPod(e.ctx, pod); err != nil {
		return nil, err
	}
	ev, err := e.ctx.Eval(0)
	if err != nil {
		return nil, err
	}
	st := &podState{ev: ev, index: make(map[string]int, len(names))}
	for i, n := range names {
		st.index[n] = i
	}
	cs.Write(stateKey, st)
	return st, nil
}

// Plugin is one in-tree plugin backed by the shared per-pod evaluation.
type Plugin struct {
	name string
	id   int
	norm bool // has ScoreExtensions (TaintToleration, NodeAffinity, PodTopologySpread, InterPodAffinity)
	ev   *Evaluator
	h    framework.Handle
}

func (p *Plugin) Name() string { return p.name }

// PreFilter runs the whole sweep for the pod (first plugin to get here pays).
func (p *Plugin) PreFilter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod) (*framework.PreFilterResult, *framework.Status) {
	all, err := p.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	st, err := p.ev.evalPod(ctx, cs, pod, all)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	_ = st
	// Skip decisions are host-decidable (encoder: filter_skip) except the
	// InterPodAffinity one reported in ev.Status (KSG_ST_IPA_PREFILTER_SKIP).
	return nil, nil
}

func (p *Plugin) PreFilterExtensions() framework.PreFilterExtensions { return nil }

// Filter answers from the stashed status word: reject iff this plugin is
// the first one that rejected the node (the framework stops there).
func (p *Plugin) Filter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	d, err := cs.Read(stateKey)
	if err != nil {
		return framework.AsStatus(err)
	}
	st := d.(*podState)
	i, ok := st.index[ni.Node().Name]
	if !ok {
		return framework.AsStatus(fmt.Errorf("node %q not in snapshot", ni.Node().Name))
	}
	w := st.ev.FStatus[i]
	if w == 0 || int(w&0xff)-1 != p.id {
		return nil
	}
	code, msg := p.ev.enc.Message(p.id, w, ni.Node().Name)
	return framework.NewStatus(code, msg)
}

func (p *Plugin) PreScore(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, nodes []*framework.NodeInfo) *framework.Status {
	d, err := cs.Read(stateKey)
	if err != nil {
		return framework.AsStatus(err)
	}
	if d.(*podState).ev.ScoreSkip&(1<<uint(p.id)) != 0 {
		return framework.NewStatus(framework.Skip)
	}
	return nil
}

// Score returns the raw Score() value computed on the device.
func (p *Plugin) Score(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, nodeName string) (int64, *framework.Status) {
	d, err := cs.Read(stateKey)
	if err != nil {
		return 0, framework.AsStatus(err)
	}
	st := d.(*podState)
	n := len(st.ev.Total)
	return st.ev.Raw[p.id*n+st.index[nodeName]], nil
}

func (p *Plugin) ScoreExtensions() framework.ScoreExtensions {
	if p.norm {
		return p
	}
	return nil
}

// NormalizeScore overwrites the list with the device's normalised values.
func (p *Plugin) NormalizeScore(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, scores framework.NodeScoreList) *framework.Status {
	d, err := cs.Read(stateKey)
	if err != nil {
		return framework.AsStatus(err)
	}
	st := d.(*podState)
	n := len(st.ev.Total)
	for k := range scores {
		scores[k].Score = st.ev.Norm[p.id*n+st.index[scores[k].Name]]
	}
	return nil
}

// Reserve assumes the pod on the device (NodeInfo.AddPod restated).
func (p *Plugin) Reserve(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, nodeName string) *framework.Status {
	d, err := cs.Read(stateKey)
	if err != nil {
		return framework.AsStatus(err)
	}
	if err := p.ev.ctx.Commit(0, d.(*podState).index[nodeName]); err != nil {
		return framework.AsStatus(err)
	}
	return nil
}

func (p *Plugin) Unreserve(ctx context.Context, cs *framework.CycleState, pod *v1.Pod, nodeName string) {}

// Factories returns in-tree-named factories sharing one Evaluator.
func Factories(ev *Evaluator) map[string]func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error) {
	mk := func(name string, id int, norm bool) func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error) {
		return func(_ context.Context, _ runtime.Object, h framework.Handle) (framework.Plugin, error) {
			return &Plugin{name: name, id: id, norm: norm, ev: ev, h: h}, nil
		}
	}
	return map[string]func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error){
		"NodeUnschedulable":  mk("NodeUnschedulable", ksched.NodeUnschedulable, false),
		"NodeName":           mk("NodeName", ksched.NodeName, false),
		"TaintToleration":    mk("TaintToleration", ksched.TaintToleration, true),
		"NodeAffinity":       mk("NodeAffinity", ksched.NodeAffinity, true),
		"NodeResourcesFit":   mk("NodeResourcesFit", ksched.NodeResourcesFit, false),
		"PodTopologySpread":  mk("PodTopologySpread", ksched.PodTopologySpread, true),
		"InterPodAffinity":   mk("InterPodAffinity", ksched.InterPodAffinity, true),
		"NodeResourcesBalancedAllocation": mk("NodeResourcesBalancedAllocation", ksched.BalancedAllocation, false),
		"ImageLocality":      mk("ImageLocality", ksched.ImageLocality, false),
	}
}
