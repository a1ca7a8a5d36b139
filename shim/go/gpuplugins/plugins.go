// Package gpuplugins exposes the MI355X evaluator as in-tree-named Scheduling
// Framework plugins, so the simulator's wrappedPlugin and resultstore.Store
// stay unchanged (SURVEY.md §8(b)).  Source only (no Go toolchain here).
//
// Wiring: overlay Factories(ev) onto the in-tree registry returned at
// simulator/scheduler/config/plugin.go:49-51 (plugins.go:50 looks in-tree up
// first), or add an option next to debuggablescheduler.WithPlugin
// (simulator/pkg/debuggablescheduler/command.go:64-68).  Name() returns the
// in-tree name, so Store keys (wrappedplugin.go:406,438,542) and
// getScorePluginWeight (plugins.go:295) see the same names as today.
//
// Each plugin implements exactly the extension points its upstream v1.32
// counterpart implements: NewWrappedPlugin type-asserts every interface
// (wrappedplugin.go:253-360) and records a result for each one it finds, so
// an extra method (a Reserve on NodeResourcesFit, say) would add an
// annotation entry the reference never writes.  Assumed pods therefore reach
// the device through the next cycle's snapshot diff (Evaluator.syncCluster),
// not through a Reserve plugin.
package gpuplugins

import (
	"context"
	"fmt"
	"sync"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/runtime"
	"k8s.io/apimachinery/pkg/types"
	"k8s.io/apimachinery/pkg/util/sets"
	"k8s.io/client-go/tools/cache"
	"k8s.io/kubernetes/pkg/scheduler/framework"

	"example.invalid/ksched-mi355x/shim/go/ksched"
)

const stateKey framework.StateKey = "ksched/eval"

const fsNotEvaluated = 0xFF // KSG_FS_NOT_EVALUATED

// podState is the per-pod SoA result, computed once per scheduling cycle,
// with every node's framework.Status and every plugin's PreFilter status
// decoded up front, so the framework's 16 Filter / Score goroutines read it
// without taking Evaluator.mu.
type podState struct {
	pod   int // snapshot pod index
	ev    *ksched.PodEval
	index map[string]int // node name -> column (the Evaluator's, built once per snapshot load)
	codes []int32        // per node: framework.Code of the rejection (ksched.Code*)
	msgID []int32        // per node: index into msgs, -1 = passed / not evaluated
	msgs  []string
	pre   [ksched.NPlugins]preFilterResult
	// nodes with nominated pods of priority >= the pod's: the node's Filter
	// verdict with those pods assumed (RunFilterPluginsWithNominatedPods' first
	// pass), and the nominated UIDs that identify that pass's NodeInfo
	nom map[int]*nominatedVerdict
}

type nominatedVerdict struct {
	word uint32
	code int32
	msg  string
	uids map[types.UID]bool
}

type preFilterResult struct {
	code  int
	names []string // NodeAffinity's / VolumeBinding's PreFilterResult, nil = none
	msg   string   // a rejection's message (ksg_snapshot_prefilter_message)
}

func (s *podState) Clone() framework.StateData { return s }

// DefaultSelectorFunc is helper.DefaultSelector over the handle's service /
// RC / RS / StatefulSet listers (PodTopologySpread system defaults); nil
// when PodTopologySpread is not system-defaulted.
type DefaultSelectorFunc func(*v1.Pod) labels.Selector

// Evaluator owns the device context and the native snapshot encoder.  The
// framework calls plugins from 16 goroutines; every device call happens
// under mu, once per pod.
type Evaluator struct {
	mu         sync.Mutex
	ctx        *ksched.Ctx
	prof       *ksched.ProfileArgs
	snap       *ksched.Snapshot
	defaultSel DefaultSelectorFunc

	nodes   []string          // column order of the loaded snapshot
	index   map[string]int    // node name -> column; replaced (never mutated) by rebuild
	nodeRV  map[string]string // node ResourceVersion at load
	nodeGen map[string]int64  // NodeInfo.Generation at the last diff
	podIdx  map[types.UID]int // pod -> snapshot index
	podRV   map[types.UID]string
	podNode map[types.UID]int // pods bound / assumed on the device -> column
	hinted  map[types.UID]struct{} // pending pods announced to this snapshot (hintPending)
	// snapshot pods no longer current (a pod re-encoded after an update, a
	// pod that left its node, a pending pod deleted): the snapshot only
	// appends, so once they outnumber the live pods (podIdx) past a threshold
	// the next sync rebuilds it from the NodeInfos (bound pods only)
	stale int

	// fed by informer handlers (attach), drained under mu:
	side      sync.Mutex
	nominated map[string]struct{} // nodes that may hold nominated pods
	subscribed bool               // attach() registered the pod informer: nominated is maintained
	gone      []*v1.Pod           // pods deleted since the last sync
	pending   []*v1.Pod           // pending pods created since the last sync (hinted to the snapshot)
	nsDirty   bool                // a namespace was added or its labels changed
	attached  sync.Once
	nsList    func() ([]*v1.Namespace, error) // the handle's namespace lister, nil before attach
	// the volume plugins' listers (PVs, claims, classes): every object is handed
	// to the snapshot when one changed (the next encode is then a full one)
	stDirty bool
	stSync  func(*ksched.Snapshot) error
}

// staleLimit: rebuild once this many superseded snapshot pods accumulated
// (and they outnumber the live ones).
const staleLimit = 4096

// NewEvaluator opens device dev for profile 0.
func NewEvaluator(dev int, prof *ksched.ProfileArgs, ds DefaultSelectorFunc) (*Evaluator, error) {
	ctx, err := ksched.Open(dev)
	if err != nil {
		return nil, err
	}
	return &Evaluator{ctx: ctx, prof: prof, defaultSel: ds, nominated: map[string]struct{}{}}, nil
}

// attach subscribes to the handle's informers once: namespaces (their labels
// resolve namespaceSelector terms: the snapshot must hold them before any pod
// that uses one is encoded) and pods (nominations, so the nominated pass
// visits only nodes that may hold nominated pods, and deletions of pending
// pods, which make their snapshot entries stale).
func (e *Evaluator) attach(h framework.Handle) {
	e.attached.Do(func() {
		f := h.SharedInformerFactory()
		if f == nil {
			return // no informers: nominatedPass visits every node (subscribed stays false)
		}
		nsInf := f.Core().V1().Namespaces()
		lister := nsInf.Lister()
		e.side.Lock()
		e.nsList = func() ([]*v1.Namespace, error) { return lister.List(labels.Everything()) }
		e.nsDirty = true
		e.side.Unlock()
		_, _ = nsInf.Informer().AddEventHandler(cache.ResourceEventHandlerFuncs{
			AddFunc:    func(interface{}) { e.markNamespaces() },
			UpdateFunc: func(o, n interface{}) { e.markNamespaces() },
		})
		pvInf, pvcInf, scInf := f.Core().V1().PersistentVolumes(), f.Core().V1().PersistentVolumeClaims(),
			f.Storage().V1().StorageClasses()
		pvL, pvcL, scL := pvInf.Lister(), pvcInf.Lister(), scInf.Lister()
		e.side.Lock()
		e.stSync = func(snap *ksched.Snapshot) error {
			scs, err := scL.List(labels.Everything())
			if err != nil {
				return err
			}
			// the listers' state replaces the snapshot's: a deleted PV / claim /
			// class leaves it (a pod naming a deleted claim is then rejected at
			// PreFilter, as upstream's lister lookup rejects it)
			if err := snap.ClearStorage(); err != nil {
				return err
			}
			for _, sc := range scs {
				if err := snap.AddStorageClass(sc); err != nil {
					return err
				}
			}
			pvs, err := pvL.List(labels.Everything())
			if err != nil {
				return err
			}
			for _, pv := range pvs {
				if err := snap.AddPV(pv); err != nil {
					return err
				}
			}
			pvcs, err := pvcL.List(labels.Everything())
			if err != nil {
				return err
			}
			for _, c := range pvcs {
				if err := snap.AddPVC(c); err != nil {
					return err
				}
			}
			return nil
		}
		e.stDirty = true
		e.side.Unlock()
		mark := cache.ResourceEventHandlerFuncs{
			AddFunc:    func(interface{}) { e.markStorage() },
			UpdateFunc: func(o, n interface{}) { e.markStorage() },
			DeleteFunc: func(interface{}) { e.markStorage() },
		}
		for _, inf := range []cache.SharedIndexInformer{pvInf.Informer(), pvcInf.Informer(), scInf.Informer()} {
			_, _ = inf.AddEventHandler(mark)
		}
		_, _ = f.Core().V1().Pods().Informer().AddEventHandler(cache.ResourceEventHandlerFuncs{
			AddFunc:    func(o interface{}) { e.notePod(o) },
			UpdateFunc: func(_, n interface{}) { e.notePod(n) },
			DeleteFunc: func(o interface{}) {
				if t, ok := o.(cache.DeletedFinalStateUnknown); ok {
					o = t.Obj
				}
				if p, ok := o.(*v1.Pod); ok {
					e.side.Lock()
					e.gone = append(e.gone, p)
					e.side.Unlock()
				}
			},
		})
		e.side.Lock()
		e.subscribed = true
		e.side.Unlock()
	})
}

func (e *Evaluator) markStorage() {
	e.side.Lock()
	e.stDirty = true
	e.side.Unlock()
}

// syncStorage (under mu) hands the PVs, claims and classes to the snapshot
// when one changed (or at a rebuild): pods with claims resolve against them.
// The snapshot's storage is cleared first, so a deleted object leaves it at
// the next sync and the claims that named it are unresolved, as upstream's
// listers would have them.
func (e *Evaluator) syncStorage(force bool) error {
	e.side.Lock()
	dirty, sync := e.stDirty || force, e.stSync
	e.stDirty = false
	e.side.Unlock()
	if !dirty || sync == nil || e.snap == nil {
		return nil
	}
	return sync(e.snap)
}

func (e *Evaluator) markNamespaces() {
	e.side.Lock()
	e.nsDirty = true
	e.side.Unlock()
}

func (e *Evaluator) notePod(o interface{}) {
	p, ok := o.(*v1.Pod)
	if !ok {
		return
	}
	if p.Status.NominatedNodeName != "" {
		e.noteNominated(p.Status.NominatedNodeName)
	}
	if p.Spec.NodeName == "" && p.DeletionTimestamp == nil {
		e.side.Lock()
		e.pending = append(e.pending, p)
		e.side.Unlock()
	}
}

// hintPending (under mu) announces the pending pods the informer delivered
// since the last sync to the snapshot (ksg_snapshot_hint_pod): a burst of new
// workloads costs one re-encode at the next sync instead of one per pod.  A
// pod the encoder refuses is left to its own cycle, which reports it.
func (e *Evaluator) hintPending() {
	e.side.Lock()
	pend := e.pending
	e.pending = nil
	e.side.Unlock()
	if e.snap == nil {
		return
	}
	if e.hinted == nil {
		e.hinted = map[types.UID]struct{}{}
	}
	for _, p := range pend {
		if _, known := e.podIdx[p.UID]; known {
			continue
		}
		if _, done := e.hinted[p.UID]; done {
			continue
		}
		e.hinted[p.UID] = struct{}{}
		_ = e.snap.HintPod(p, e.selectorOf(p))
	}
}

// noteNominated records a node that may hold nominated pods (the informer,
// and this shim's own PostFilter when it nominates).
func (e *Evaluator) noteNominated(node string) {
	e.side.Lock()
	e.nominated[node] = struct{}{}
	e.side.Unlock()
}

// syncNamespaces (under mu) registers every namespace with the snapshot when
// one was added or relabelled since the last sync; the native encoder
// re-resolves namespaceSelector terms when a namespace's labels change.
func (e *Evaluator) syncNamespaces(force bool) error {
	e.side.Lock()
	dirty, list := e.nsDirty || force, e.nsList
	e.nsDirty = false
	e.side.Unlock()
	if !dirty || list == nil || e.snap == nil {
		return nil
	}
	nss, err := list()
	if err != nil {
		return err
	}
	for _, ns := range nss {
		if err := e.snap.AddNamespace(ns); err != nil {
			return err
		}
	}
	return nil
}

// pruneGone (under mu) drops pods deleted while pending from the maps and
// counts their snapshot entries as stale.
func (e *Evaluator) pruneGone() {
	e.side.Lock()
	gone := e.gone
	e.gone = nil
	e.side.Unlock()
	for _, p := range gone {
		uid := p.UID
		if _, ok := e.hinted[uid]; ok { // a pending pod deleted before its cycle: its hint goes too
			delete(e.hinted, uid)
			if e.snap != nil {
				_ = e.snap.UnhintPod(p.Namespace, p.Name)
			}
		}
		if c, ok := e.podNode[uid]; ok && c >= 0 {
			continue // still on the device: syncCluster forgets it when it leaves its node
		}
		if _, ok := e.podIdx[uid]; ok {
			e.forgetUID(uid)
		}
	}
}

func (e *Evaluator) forgetUID(uid types.UID) {
	delete(e.podIdx, uid)
	delete(e.podRV, uid)
	delete(e.podNode, uid)
	e.stale++
}

func (e *Evaluator) selectorOf(p *v1.Pod) labels.Selector {
	if e.defaultSel == nil {
		return nil
	}
	return e.defaultSel(p)
}

// rebuild encodes the whole snapshot: every node, every pod on them (bound),
// then loads it (bindings replayed as assumes).
func (e *Evaluator) rebuild(infos []*framework.NodeInfo) error {
	if e.snap != nil {
		e.snap.Free()
	}
	snap, err := ksched.NewSnapshot(e.prof)
	if err != nil {
		return err
	}
	e.snap = snap
	e.nodes = e.nodes[:0]
	e.index = make(map[string]int, len(infos))
	e.nodeRV, e.nodeGen = map[string]string{}, map[string]int64{}
	e.podIdx, e.podRV, e.podNode = map[types.UID]int{}, map[types.UID]string{}, map[types.UID]int{}
	e.stale = 0
	e.hinted = nil // a new snapshot: pending pods are announced again as they arrive
	for col, ni := range infos {
		n := ni.Node()
		if _, err := snap.AddNode(n); err != nil {
			return err
		}
		e.nodes = append(e.nodes, n.Name)
		e.index[n.Name] = col
		e.nodeRV[n.Name] = n.ResourceVersion
		e.nodeGen[n.Name] = ni.Generation
	}
	// every namespace before the first pod: a bound pod's namespaceSelector
	// term needs them to encode
	if err := e.syncStorage(true); err != nil {
		return err
	}
	if err := e.syncNamespaces(true); err != nil {
		return err
	}
	for col, ni := range infos {
		for _, pi := range ni.Pods {
			idx, err := snap.AddPod(pi.Pod, e.selectorOf(pi.Pod))
			if err != nil {
				return err
			}
			if err := snap.Bind(idx, col); err != nil {
				return err
			}
			e.podIdx[pi.Pod.UID], e.podRV[pi.Pod.UID], e.podNode[pi.Pod.UID] = idx, pi.Pod.ResourceVersion, col
		}
	}
	return snap.Load(e.ctx)
}

// syncCluster brings the device up to date with the framework's snapshot:
// a changed node set or node object reloads everything; otherwise the pods
// that appeared on / left a node since the last cycle (the previous cycle's
// assume among them) are assumed / forgotten one by one.
func (e *Evaluator) syncCluster(infos []*framework.NodeInfo) error {
	e.pruneGone()
	same := e.snap != nil && len(infos) == len(e.nodes) &&
		!(e.stale > staleLimit && e.stale > len(e.podIdx))
	for i := 0; same && i < len(infos); i++ {
		n := infos[i].Node()
		same = n.Name == e.nodes[i] && n.ResourceVersion == e.nodeRV[n.Name]
	}
	if !same {
		return e.rebuild(infos)
	}
	if err := e.syncStorage(false); err != nil {
		return err
	}
	if err := e.syncNamespaces(false); err != nil {
		return err
	}
	e.hintPending()
	for col, ni := range infos {
		name := e.nodes[col]
		if ni.Generation == e.nodeGen[name] {
			continue
		}
		present := make(map[types.UID]bool, len(ni.Pods))
		for _, pi := range ni.Pods {
			uid := pi.Pod.UID
			present[uid] = true
			if c, ok := e.podNode[uid]; ok && c == col {
				continue
			}
			idx, known := e.podIdx[uid]
			if known && e.podRV[uid] != pi.Pod.ResourceVersion && e.podNode[uid] >= 0 {
				return e.rebuild(infos) // a bound pod changed: re-encode
			}
			if !known {
				var err error
				if idx, err = e.snap.AddPod(pi.Pod, e.selectorOf(pi.Pod)); err != nil {
					return err
				}
				if _, err := e.snap.Sync(e.ctx); err != nil {
					return err
				}
				e.podIdx[uid], e.podRV[uid] = idx, pi.Pod.ResourceVersion
			}
			if c, ok := e.podNode[uid]; ok && c >= 0 {
				if err := e.snap.Forget(e.ctx, idx, c); err != nil {
					return err
				}
			}
			if err := e.snap.Assume(e.ctx, idx, col); err != nil {
				return err
			}
			e.podNode[uid] = col
		}
		for uid, c := range e.podNode {
			if c == col && !present[uid] {
				if err := e.snap.Forget(e.ctx, e.podIdx[uid], col); err != nil {
					return err
				}
				// deleted (or moved: a node visited later finds it unknown and
				// encodes it afresh); its snapshot entry is stale either way
				e.forgetUID(uid)
			}
		}
		e.nodeGen[name] = ni.Generation
	}
	return nil
}

// evalPod runs the whole sweep for the pod once per cycle (the first of the
// shim's plugins to be called pays) and stashes it in CycleState.
func (e *Evaluator) evalPod(cs *framework.CycleState, pod *v1.Pod, infos []*framework.NodeInfo,
	nom framework.PodNominator) (*podState, error) {
	if d, err := cs.Read(stateKey); err == nil {
		return d.(*podState), nil
	}
	e.mu.Lock()
	defer e.mu.Unlock()
	if err := e.syncCluster(infos); err != nil {
		return nil, err
	}
	idx, known := e.podIdx[pod.UID]
	if known && e.podRV[pod.UID] != pod.ResourceVersion {
		known = false // the pod object changed since it was encoded: encode it again
		e.stale++
	}
	if !known {
		var err error
		if idx, err = e.snap.AddPod(pod, e.selectorOf(pod)); err != nil {
			return nil, err
		}
		e.podIdx[pod.UID], e.podRV[pod.UID] = idx, pod.ResourceVersion
		if _, ok := e.podNode[pod.UID]; !ok {
			e.podNode[pod.UID] = -1
		}
	}
	if _, err := e.snap.Sync(e.ctx); err != nil {
		return nil, err
	}
	if pod.Status.NominatedNodeName != "" {
		e.noteNominated(pod.Status.NominatedNodeName)
	}
	st := &podState{pod: idx, index: e.index}
	// nominated pods first: their evaluations reuse the library's result
	// block, which the pod's own evaluation below then keeps for the cycle
	if nom != nil {
		if err := e.nominatedPass(st, pod, nom); err != nil {
			return nil, err
		}
	}
	ev, err := e.ctx.EvalView(idx)
	if err != nil {
		return nil, err
	}
	st.ev = ev
	// every rejected node's Status, once per pod (ksg_snapshot_statuses)
	if st.codes, st.msgID, st.msgs, err = e.snap.Statuses(idx, ev.FStatus); err != nil {
		return nil, err
	}
	for id := 0; id < ksched.NPlugins; id++ {
		code, names, err := e.snap.PreFilter(idx, id, ev.Status)
		if err != nil {
			return nil, err
		}
		msg := ""
		if code == ksched.CodeUnschedulableAndUnresolvable {
			if msg, err = e.snap.PreFilterMessage(idx, id); err != nil {
				return nil, err
			}
		}
		st.pre[id] = preFilterResult{code: code, names: names, msg: msg}
	}
	cs.Write(stateKey, st)
	return st, nil
}

// nominatedPass restates addGENominatedPods + RunFilterPluginsWithNominatedPods
// [framework/runtime/framework.go, v1.32]: for each node holding nominated
// pods of priority >= the pod's (other than the pod itself), evaluate once
// more with only that node's nominated pods assumed on it (PreFilter state
// and NodeInfo both see them, as AddPod extensions would), then forget them.
// Filter answers the framework's first pass from this verdict and its second
// pass from the plain evaluation.  Nominated nodes are few (preemptors
// waiting for their victims to leave), so this costs an evaluation each.
// Only nodes that may hold nominated pods are visited (attach, PostFilter);
// a node found without any is dropped from that set.
func (e *Evaluator) nominatedPass(st *podState, pod *v1.Pod, nom framework.PodNominator) error {
	prio := podPriority(pod)
	e.side.Lock()
	names := make([]string, 0, len(e.nominated))
	if e.subscribed {
		for name := range e.nominated {
			names = append(names, name)
		}
	} else { // nobody reports nominations to this evaluator: every node may hold some
		for name := range e.index {
			names = append(names, name)
		}
	}
	e.side.Unlock()
	for _, name := range names {
		col, ok := e.index[name]
		nominated := nom.NominatedPodsForNode(name)
		if len(nominated) == 0 {
			e.side.Lock()
			delete(e.nominated, name)
			e.side.Unlock()
		}
		if !ok {
			continue
		}
		var add []*v1.Pod
		for _, pi := range nominated {
			if pi.Pod.UID != pod.UID && podPriority(pi.Pod) >= prio {
				add = append(add, pi.Pod)
			}
		}
		if len(add) == 0 {
			continue
		}
		v := &nominatedVerdict{uids: map[types.UID]bool{}}
		var assumed []int
		forget := func() error {
			for _, q := range assumed {
				if err := e.snap.Forget(e.ctx, q, col); err != nil {
					return err
				}
			}
			return nil
		}
		for _, q := range add {
			idx, known := e.podIdx[q.UID]
			if !known || e.podRV[q.UID] != q.ResourceVersion {
				if known {
					e.stale++
				}
				var err error
				if idx, err = e.snap.AddPod(q, e.selectorOf(q)); err != nil {
					_ = forget()
					return err
				}
				if _, err := e.snap.Sync(e.ctx); err != nil {
					_ = forget()
					return err
				}
				e.podIdx[q.UID], e.podRV[q.UID] = idx, q.ResourceVersion
				if _, ok := e.podNode[q.UID]; !ok {
					e.podNode[q.UID] = -1
				}
			}
			if err := e.snap.Assume(e.ctx, idx, col); err != nil {
				_ = forget()
				return err
			}
			assumed = append(assumed, idx)
			v.uids[q.UID] = true
		}
		ev, err := e.ctx.Eval(st.pod)
		if ferr := forget(); err == nil {
			err = ferr
		}
		if err != nil {
			return err
		}
		v.word = ev.FStatus[col]
		if v.word != 0 && v.word != fsNotEvaluated {
			code, msg, err := e.snap.Status(st.pod, v.word, col)
			if err != nil {
				return err
			}
			v.code, v.msg = int32(code), msg
		}
		if st.nom == nil {
			st.nom = map[int]*nominatedVerdict{}
		}
		st.nom[col] = v
	}
	return nil
}

// podPriority is corev1helpers.PodPriority.
func podPriority(p *v1.Pod) int32 {
	if p.Spec.Priority != nil {
		return *p.Spec.Priority
	}
	return 0
}

// status answers one Filter call from the pod's decoded statuses (no lock).
// ni is the NodeInfo the framework filters against: on a node with
// nominated pods, the first pass's NodeInfo holds them and is answered from
// the nominated verdict.
func (e *Evaluator) status(st *podState, id int, ni *framework.NodeInfo) *framework.Status {
	node := ni.Node().Name
	col, ok := st.index[node]
	if !ok {
		return framework.AsStatus(fmt.Errorf("node %q not in the evaluated snapshot", node))
	}
	if v := st.nom[col]; v != nil {
		for _, pi := range ni.Pods {
			if v.uids[pi.Pod.UID] {
				if v.word == 0 || v.word == fsNotEvaluated || int(v.word&0xff)-1 != id {
					return nil
				}
				return framework.NewStatus(frameworkCode(int(v.code)), v.msg)
			}
		}
	}
	w := st.ev.FStatus[col]
	if w == 0 || w == fsNotEvaluated || int(w&0xff)-1 != id {
		return nil // passed this plugin (the framework stops at the first rejection, as the device does)
	}
	return framework.NewStatus(frameworkCode(int(st.codes[col])), st.msgs[st.msgID[col]])
}

// applyArgs records a factory's decoded args; a change after the snapshot
// was built re-encodes it at the next cycle.
func (e *Evaluator) applyArgs(name string, obj runtime.Object) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	if err := e.prof.ApplyPluginArgs(name, obj); err != nil {
		return err
	}
	if e.snap != nil {
		e.snap.Free()
		e.snap = nil
		e.nodes = nil
	}
	return nil
}

func frameworkCode(c int) framework.Code {
	switch c {
	case ksched.CodeSuccess:
		return framework.Success
	case ksched.CodeUnschedulable:
		return framework.Unschedulable
	case ksched.CodeUnschedulableAndUnresolvable:
		return framework.UnschedulableAndUnresolvable
	case ksched.CodeSkip:
		return framework.Skip
	}
	return framework.Error
}

// ---- plugin bodies shared by the per-extension-point types below ------------

type base struct {
	name string
	id   int
	ev   *Evaluator
	h    framework.Handle
}

func (b *base) Name() string { return b.name }

func (b *base) state(cs *framework.CycleState) (*podState, *framework.Status) {
	d, err := cs.Read(stateKey)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	return d.(*podState), nil
}

// run makes sure the pod was evaluated (plugins without a PreFilter can be
// the first of the shim's plugins the framework calls).
func (b *base) run(cs *framework.CycleState, pod *v1.Pod) (*podState, *framework.Status) {
	if st, s := b.state(cs); s == nil {
		return st, nil
	}
	infos, err := b.h.SnapshotSharedLister().NodeInfos().List()
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	st, err := b.ev.evalPod(cs, pod, infos, b.h)
	if err != nil {
		return nil, framework.AsStatus(err)
	}
	return st, nil
}

func (b *base) preFilter(cs *framework.CycleState, pod *v1.Pod) (*framework.PreFilterResult, *framework.Status) {
	st, s := b.run(cs, pod)
	if s != nil {
		return nil, s
	}
	code, names := st.pre[b.id].code, st.pre[b.id].names
	switch code {
	case ksched.CodeSkip:
		return nil, framework.NewStatus(framework.Skip) // recorded as "" (store.go:522)
	case ksched.CodeUnschedulableAndUnresolvable: // nodeaffinity errReasonConflict
		return nil, framework.NewStatus(framework.UnschedulableAndUnresolvable, st.pre[b.id].msg)
	}
	if names != nil {
		return &framework.PreFilterResult{NodeNames: sets.New[string](names...)}, nil
	}
	return nil, nil
}

func (b *base) filter(cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	st, s := b.run(cs, pod)
	if s != nil {
		return s
	}
	return b.ev.status(st, b.id, ni)
}

func (b *base) preScore(cs *framework.CycleState, pod *v1.Pod) *framework.Status {
	st, s := b.run(cs, pod)
	if s != nil {
		return s
	}
	if st.ev.ScoreSkip&(1<<uint(b.id)) != 0 {
		return framework.NewStatus(framework.Skip)
	}
	return nil
}

func (b *base) score(cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	st, s := b.run(cs, pod)
	if s != nil {
		return 0, s
	}
	return st.ev.Raw(b.id, st.index[node]), nil
}

func (b *base) normalize(cs *framework.CycleState, scores framework.NodeScoreList) *framework.Status {
	st, s := b.state(cs)
	if s != nil {
		return s
	}
	for k := range scores {
		scores[k].Score = st.ev.Norm(b.id, st.index[scores[k].Name])
	}
	return nil
}

// ---- one type per upstream extension-point set ---------------------------

// filterOnly: NodeUnschedulable, NodeName.
type filterOnly struct{ base }

func (p *filterOnly) Filter(_ context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	return p.filter(cs, pod, ni)
}

// taintToleration: Filter, PreScore, Score + NormalizeScore.
type taintToleration struct{ base }

func (p *taintToleration) Filter(_ context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	return p.filter(cs, pod, ni)
}
func (p *taintToleration) PreScore(_ context.Context, cs *framework.CycleState, pod *v1.Pod, _ []*framework.NodeInfo) *framework.Status {
	return p.preScore(cs, pod)
}
func (p *taintToleration) Score(_ context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	return p.score(cs, pod, node)
}
func (p *taintToleration) ScoreExtensions() framework.ScoreExtensions { return p }
func (p *taintToleration) NormalizeScore(_ context.Context, cs *framework.CycleState, _ *v1.Pod, s framework.NodeScoreList) *framework.Status {
	return p.normalize(cs, s)
}

// allPoints: NodeAffinity, PodTopologySpread, InterPodAffinity.
type allPoints struct{ base }

func (p *allPoints) PreFilter(_ context.Context, cs *framework.CycleState, pod *v1.Pod) (*framework.PreFilterResult, *framework.Status) {
	return p.preFilter(cs, pod)
}
func (p *allPoints) PreFilterExtensions() framework.PreFilterExtensions { return nil }
func (p *allPoints) Filter(_ context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	return p.filter(cs, pod, ni)
}
func (p *allPoints) PreScore(_ context.Context, cs *framework.CycleState, pod *v1.Pod, _ []*framework.NodeInfo) *framework.Status {
	return p.preScore(cs, pod)
}
func (p *allPoints) Score(_ context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	return p.score(cs, pod, node)
}
func (p *allPoints) ScoreExtensions() framework.ScoreExtensions { return p }
func (p *allPoints) NormalizeScore(_ context.Context, cs *framework.CycleState, _ *v1.Pod, s framework.NodeScoreList) *framework.Status {
	return p.normalize(cs, s)
}

// fit: NodeResourcesFit (PreFilter, Filter, PreScore, Score; no normalise).
type fit struct{ base }

func (p *fit) PreFilter(_ context.Context, cs *framework.CycleState, pod *v1.Pod) (*framework.PreFilterResult, *framework.Status) {
	return p.preFilter(cs, pod)
}
func (p *fit) PreFilterExtensions() framework.PreFilterExtensions { return nil }
func (p *fit) Filter(_ context.Context, cs *framework.CycleState, pod *v1.Pod, ni *framework.NodeInfo) *framework.Status {
	return p.filter(cs, pod, ni)
}
func (p *fit) PreScore(_ context.Context, cs *framework.CycleState, pod *v1.Pod, _ []*framework.NodeInfo) *framework.Status {
	return p.preScore(cs, pod)
}
func (p *fit) Score(_ context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	return p.score(cs, pod, node)
}
func (p *fit) ScoreExtensions() framework.ScoreExtensions { return nil }

// balanced: NodeResourcesBalancedAllocation (PreScore, Score).
type balanced struct{ base }

func (p *balanced) PreScore(_ context.Context, cs *framework.CycleState, pod *v1.Pod, _ []*framework.NodeInfo) *framework.Status {
	return p.preScore(cs, pod)
}
func (p *balanced) Score(_ context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	return p.score(cs, pod, node)
}
func (p *balanced) ScoreExtensions() framework.ScoreExtensions { return nil }

// imageLocality: Score only.
type imageLocality struct{ base }

func (p *imageLocality) Score(_ context.Context, cs *framework.CycleState, pod *v1.Pod, node string) (int64, *framework.Status) {
	return p.score(cs, pod, node)
}
func (p *imageLocality) ScoreExtensions() framework.ScoreExtensions { return nil }

// Factories returns in-tree-named factories sharing one Evaluator (the
// PluginFactory signature of k8s.io/kubernetes v1.32 runtime.Registry).
func Factories(ev *Evaluator) map[string]func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error) {
	type mk func(b base) framework.Plugin
	table := []struct {
		name string
		id   int
		make mk
	}{
		{"NodeUnschedulable", ksched.NodeUnschedulable, func(b base) framework.Plugin { return &filterOnly{b} }},
		{"NodeName", ksched.NodeName, func(b base) framework.Plugin { return &filterOnly{b} }},
		{"TaintToleration", ksched.TaintToleration, func(b base) framework.Plugin { return &taintToleration{b} }},
		{"NodeAffinity", ksched.NodeAffinity, func(b base) framework.Plugin { return &allPoints{b} }},
		{"NodeResourcesFit", ksched.NodeResourcesFit, func(b base) framework.Plugin { return &fit{b} }},
		{"PodTopologySpread", ksched.PodTopologySpread, func(b base) framework.Plugin { return &allPoints{b} }},
		{"InterPodAffinity", ksched.InterPodAffinity, func(b base) framework.Plugin { return &allPoints{b} }},
		{"NodeResourcesBalancedAllocation", ksched.BalancedAllocation, func(b base) framework.Plugin { return &balanced{b} }},
		{"ImageLocality", ksched.ImageLocality, func(b base) framework.Plugin { return &imageLocality{b} }},
	}
	out := map[string]func(context.Context, runtime.Object, framework.Handle) (framework.Plugin, error){}
	for _, t := range table {
		t := t
		out[t.name] = func(_ context.Context, obj runtime.Object, h framework.Handle) (framework.Plugin, error) {
			// the plugin's args as the framework decoded them (NodeResourcesFitArgs,
			// NodeResourcesBalancedAllocationArgs, InterPodAffinityArgs,
			// PodTopologySpreadArgs, NodeAffinityArgs): into the profile the
			// snapshot is encoded with
			if err := ev.applyArgs(t.name, obj); err != nil {
				return nil, err
			}
			ev.attach(h)
			return t.make(base{name: t.name, id: t.id, ev: ev, h: h}), nil
		}
	}
	return out
}
