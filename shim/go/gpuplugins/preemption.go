// DefaultPreemption on the device dry run (ksg_preempt_victims).
//
// Upstream DefaultPreemption [k8s.io/kubernetes v1.32.5
// pkg/scheduler/framework/plugins/defaultpreemption, framework/preemption;
// not vendored] re-runs every Filter plugin on a copy of each candidate node
// with the victims removed (RunFilterPluginsWithNominatedPods).  The shim's
// Filter answers from the pod's device result for the unmodified node, so
// the upstream plugin cannot be kept: this PostFilter replaces it under the
// same name, with the steps of kube-scheduler-simulator_amd/preemption.py
// (the Python mirror the GPU tests pin against the oracle and the
// independent restatement):
//  1. PodEligibleToPreemptOthers (preemptionPolicy Never);
//  2. potential nodes = Unschedulable (not UnschedulableAndUnresolvable)
//     filter statuses, from the device's status words;
//  3. SelectVictimsOnNode for all of them in one ksg_preempt_victims call
//     (Fit, NodePorts, and PodTopologySpread / InterPodAffinity with the
//     victims' domain counts moved, for preemptors with topology terms), on
//     the nodes whose node-static filters pass (ksg_eval_skipping with those
//     four skipped: VolumeBinding / VolumeZone ordered after Fit), after the
//     ReadWriteOncePod holders decided what no removal can clear
//     (preemption.rwop_outcome);
//  4. the first calculateNumCandidates candidates in node order,
//     pickOneNodeForPreemption's criteria, lowest column on a final tie;
//  5. prepareCandidate: delete the victims through the API (their deletion
//     events reach the device through the next cycle's snapshot diff).
// The wrapper records the nominated node (wrappedplugin.go:550-583,
// store.go:442-458) exactly as for the upstream plugin.
package gpuplugins

import (
	"context"
	"fmt"
	"math"
	"sort"

	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/kubernetes/pkg/scheduler/framework"

	"example.invalid/ksched-mi355x/shim/go/ksched"
)

// PreemptionArgs are DefaultPreemptionArgs (v1 defaults 10 / 100).
type PreemptionArgs struct {
	MinCandidateNodesPercentage, MinCandidateNodesAbsolute int32
}

type preemption struct {
	base
	args PreemptionArgs
}

func podPriority(p *v1.Pod) int32 {
	if p.Spec.Priority != nil {
		return *p.Spec.Priority
	}
	return 0
}

func startTime(p *v1.Pod) int64 { // util.GetPodStartTime: now when unset
	if p.Status.StartTime != nil {
		return p.Status.StartTime.UnixNano()
	}
	return math.MaxInt64
}

// moreImportant is util.MoreImportantPod (namespace/name on a full tie).
func moreImportant(a, b *v1.Pod) bool {
	if pa, pb := podPriority(a), podPriority(b); pa != pb {
		return pa > pb
	}
	if sa, sb := startTime(a), startTime(b); sa != sb {
		return sa < sb
	}
	if a.Namespace != b.Namespace {
		return a.Namespace < b.Namespace
	}
	return a.Name < b.Name
}

type candidate struct {
	col     int
	node    string
	victims []*v1.Pod // most important first
}

// pickOne is pickOneNodeForPreemption without PodDisruptionBudgets.
func pickOne(cands []candidate) candidate {
	score := []func(c candidate) int64{
		func(c candidate) int64 { return -int64(podPriority(c.victims[0])) },
		func(c candidate) int64 {
			var s int64
			for _, v := range c.victims {
				s += int64(podPriority(v)) + math.MaxInt32 + 1
			}
			return -s
		},
		func(c candidate) int64 { return -int64(len(c.victims)) },
		func(c candidate) int64 { // latest start of the highest-priority victims
			top, best := podPriority(c.victims[0]), startTime(c.victims[0])
			for _, v := range c.victims {
				if podPriority(v) == top && startTime(v) < best {
					best = startTime(v)
				}
			}
			return best
		},
	}
	pool := cands
	for _, f := range score {
		best := int64(math.MinInt64)
		for _, c := range pool {
			if v := f(c); v > best {
				best = v
			}
		}
		var next []candidate
		for _, c := range pool {
			if f(c) == best {
				next = append(next, c)
			}
		}
		pool = next
		if len(pool) == 1 {
			break
		}
	}
	return pool[0] // pool keeps column order: lowest column on a final tie
}

func (p *preemption) PostFilter(ctx context.Context, cs *framework.CycleState, pod *v1.Pod,
	_ framework.NodeToStatusReader) (*framework.PostFilterResult, *framework.Status) {
	if pod.Spec.PreemptionPolicy != nil && *pod.Spec.PreemptionPolicy == v1.PreemptNever {
		return nil, framework.NewStatus(framework.Unschedulable, "not eligible due to preemptionPolicy=Never.")
	}
	st, s := p.state(cs)
	if s != nil {
		return nil, s
	}
	infos, err := p.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	e := p.ev
	e.mu.Lock()
	defer e.mu.Unlock()
	prio := podPriority(pod)
	var potential int
	var lists []candidate
	for col, ni := range infos {
		w := st.ev.FStatus[col]
		if w == 0 || w == fsNotEvaluated {
			continue
		}
		code, _, err := e.snap.Status(st.pod, w, col)
		if err != nil {
			return nil, framework.AsStatus(err)
		}
		if code != ksched.CodeUnschedulable {
			continue // preemption cannot help on this node
		}
		potential++
		var low []*v1.Pod
		for _, pi := range ni.Pods {
			if podPriority(pi.Pod) < prio {
				low = append(low, pi.Pod)
			}
		}
		if len(low) == 0 {
			continue
		}
		sort.Slice(low, func(i, j int) bool { return moreImportant(low[i], low[j]) })
		lists = append(lists, candidate{col: col, node: ni.Node().Name, victims: low})
	}
	if len(lists) == 0 {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: 0/"+fmt.Sprint(len(infos))+" nodes are available")
	}
	if out, s := p.rwopOutcome(pod, infos, prio); s != nil {
		return nil, s
	} else if out < 0 {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: no candidate node")
	}
	// node-static verdict: the dry run re-runs only the four filters removals
	// change; a static one ordered after the recorded rejection stays failed
	fs, err := e.ctx.EvalSkipping(st.pod, staticSkip)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	kept := lists[:0]
	for _, c := range lists {
		if fs[c.col] == 0 {
			kept = append(kept, c)
		}
	}
	if lists = kept; len(lists) == 0 {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: no candidate node")
	}
	cand, off, vic := make([]int32, 0, len(lists)), []int32{0}, []int32{}
	for _, c := range lists {
		cand = append(cand, int32(c.col))
		for _, v := range c.victims {
			idx, ok := e.podIdx[v.UID]
			if !ok {
				return nil, framework.AsStatus(fmt.Errorf("victim %s/%s not in the snapshot", v.Namespace, v.Name))
			}
			vic = append(vic, int32(idx))
		}
		off = append(off, int32(len(vic)))
	}
	fits, victim, err := e.ctx.PreemptVictims(st.pod, cand, off, vic)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	want := int(int32(potential) * p.args.MinCandidateNodesPercentage / 100)
	if want < int(p.args.MinCandidateNodesAbsolute) {
		want = int(p.args.MinCandidateNodesAbsolute)
	}
	if want > potential {
		want = potential
	}
	var cands []candidate
	for k, c := range lists {
		if fits[k] == 0 {
			continue
		}
		var chosen []*v1.Pod
		for i, v := range c.victims {
			if victim[int(off[k])+i] != 0 {
				chosen = append(chosen, v)
			}
		}
		if len(chosen) == 0 {
			continue
		}
		cands = append(cands, candidate{col: c.col, node: c.node, victims: chosen})
		if len(cands) >= want {
			break
		}
	}
	if len(cands) == 0 {
		return nil, framework.NewStatus(framework.Unschedulable, "preemption: no candidate node")
	}
	best := pickOne(cands)
	e.noteNominated(best.node) // the next cycles' nominated pass visits it
	for _, v := range best.victims { // prepareCandidate
		if err := p.h.ClientSet().CoreV1().Pods(v.Namespace).Delete(ctx, v.Name, metav1.DeleteOptions{}); err != nil {
			return nil, framework.AsStatus(err)
		}
	}
	return &framework.PostFilterResult{NominatingInfo: &framework.NominatingInfo{
		NominatedNodeName: best.node, NominatingMode: framework.ModeOverride}}, framework.NewStatus(framework.Success)
}

// staticSkip: the filters SelectVictimsOnNode's removals can change.
const staticSkip = uint32(1)<<ksched.NodeResourcesFit | uint32(1)<<ksched.NodePorts |
	uint32(1)<<ksched.PodTopologySpread | uint32(1)<<ksched.InterPodAffinity

// rwopOutcome is preemption.rwop_outcome: the pods holding one of pod's
// ReadWriteOncePod claims (VolumeRestrictions' conflictingPVCRefCount).
// Removing victims clears the conflict only on a node that runs every holder
// with each of lower priority; otherwise no candidate exists (-1).  That one
// node is refused (an Error status): the dry run does not keep the holders
// evicted through the reprieve.  0: no holder.
func (p *preemption) rwopOutcome(pod *v1.Pod, infos []*framework.NodeInfo, prio int32) (int, *framework.Status) {
	f := p.h.SharedInformerFactory()
	if f == nil {
		return 0, nil
	}
	pvcs := f.Core().V1().PersistentVolumeClaims().Lister().PersistentVolumeClaims(pod.Namespace)
	rwop := map[string]struct{}{}
	for _, vol := range pod.Spec.Volumes {
		if vol.PersistentVolumeClaim == nil {
			continue
		}
		c, err := pvcs.Get(vol.PersistentVolumeClaim.ClaimName)
		if err != nil {
			continue // a missing claim is VolumeRestrictions' PreFilter rejection
		}
		for _, m := range c.Spec.AccessModes {
			if m == v1.ReadWriteOncePod {
				rwop[c.Name] = struct{}{}
			}
		}
	}
	if len(rwop) == 0 {
		return 0, nil
	}
	holderNode, holders := "", 0
	for _, ni := range infos {
		for _, pi := range ni.Pods {
			q := pi.Pod
			if q.UID == pod.UID || q.Namespace != pod.Namespace {
				continue
			}
			for _, vol := range q.Spec.Volumes {
				if vol.PersistentVolumeClaim == nil {
					continue
				}
				if _, ok := rwop[vol.PersistentVolumeClaim.ClaimName]; !ok {
					continue
				}
				if podPriority(q) >= prio || (holders > 0 && holderNode != ni.Node().Name) {
					return -1, nil
				}
				holderNode, holders = ni.Node().Name, holders+1
				break
			}
		}
	}
	if holders == 0 {
		return 0, nil
	}
	return 0, framework.AsStatus(fmt.Errorf("DefaultPreemption: a lower-priority pod on %s holds a ReadWriteOncePod claim of %s/%s (not modelled)",
		holderNode, pod.Namespace, pod.Name))
}

// PreemptionFactory returns the DefaultPreemption replacement (register it
// under "DefaultPreemption" next to Factories).
func PreemptionFactory(ev *Evaluator, args PreemptionArgs) func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error) {
	return func(_ context.Context, _ runtime.Object, h framework.Handle) (framework.Plugin, error) {
		return &preemption{base: base{name: "DefaultPreemption", ev: ev, h: h}, args: args}, nil
	}
}
