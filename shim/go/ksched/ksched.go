// Package ksched is the cgo binding of libksched.so (include/ksched.h) for the
// debuggable scheduler in simulator/scheduler.  Source only: this image has no
// Go toolchain, so it is not compiled here (DESIGN.md §1).
//
// Build: CGO_ENABLED=1, CGO_CFLAGS=-I<repo>/include,
// CGO_LDFLAGS="-L<repo>/kube-scheduler-simulator_amd -lksched -Wl,-rpath,<dir>".
package ksched

/*
#cgo LDFLAGS: -lksched
#include <stdlib.h>
#include "ksched.h"
*/
import "C"

import (
	"fmt"
	"sync"
	"unsafe"
)

// Plugin ids, identical to include/ksched.h.
const (
	NodeUnschedulable  = C.KSG_PL_NODE_UNSCHEDULABLE
	NodeName           = C.KSG_PL_NODE_NAME
	TaintToleration    = C.KSG_PL_TAINT_TOLERATION
	NodeAffinity       = C.KSG_PL_NODE_AFFINITY
	NodePorts          = C.KSG_PL_NODE_PORTS
	NodeResourcesFit   = C.KSG_PL_NODE_RESOURCES_FIT
	PodTopologySpread  = C.KSG_PL_POD_TOPOLOGY_SPREAD
	InterPodAffinity   = C.KSG_PL_INTER_POD_AFFINITY
	BalancedAllocation = C.KSG_PL_BALANCED_ALLOCATION
	ImageLocality      = C.KSG_PL_IMAGE_LOCALITY
	NPlugins           = C.KSG_NPLUGINS
)

// Error carries a KSG_E_* code and the context's message.
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("ksched: %d: %s", e.Code, e.Msg) }

// Ctx owns one device context.  Calls are serialised (a ksg_ctx is not
// thread-safe, and the framework calls plugins from 16 goroutines).
type Ctx struct {
	mu  sync.Mutex
	c   *C.ksg_ctx
	nN  int
}

func (x *Ctx) check(rc C.int) error {
	if rc == 0 {
		return nil
	}
	return &Error{Code: int(rc), Msg: C.GoString(C.ksg_last_error(x.c))}
}

// Open creates a context on HIP device dev.
func Open(dev int) (*Ctx, error) {
	x := &Ctx{}
	if rc := C.ksg_open(C.int(dev), &x.c); rc != 0 {
		return nil, &Error{Code: int(rc), Msg: "ksg_open"}
	}
	return x, nil
}

// Close releases the device context.
func (x *Ctx) Close() error {
	x.mu.Lock()
	defer x.mu.Unlock()
	rc := C.ksg_close(x.c)
	x.c = nil
	return x.check(rc)
}

// Nodes is the SoA snapshot produced by the encoder (see encoder.py for the
// column rules); Go slices are passed without copying for the duration of
// the call only (cgo pointer rules: ksched copies them).
type Nodes struct {
	NNodes, NRes                  int
	Alloc, Requested, Nonzero     []int64
	AllowedPods, PodCount         []int32
	Unschedulable                 []uint8
	NLabelCols                    int
	LabelVal                      []uint32
	LabelNum                      []int64
	LabelNumOK                    []uint8
	MaxTaints                     int
	Taints                        []uint32
	TaintEffect                   []uint8
	MaxImages                     int
	Images                        []uint32
	NImages                       int
}

func p64(s []int64) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&s[0]))
}
func p32(s []int32) *C.int32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.int32_t)(unsafe.Pointer(&s[0]))
}
func pu32(s []uint32) *C.uint32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&s[0]))
}
func pu8(s []uint8) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&s[0]))
}

// LoadNodes uploads the snapshot (topology tables may be nil when neither
// PodTopologySpread nor InterPodAffinity is enabled).
func (x *Ctx) LoadNodes(n *Nodes, topo *C.ksg_topology) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	cn := C.ksg_nodes{
		n_nodes: C.int32_t(n.NNodes), n_res: C.int32_t(n.NRes),
		alloc: p64(n.Alloc), requested: p64(n.Requested), nonzero: p64(n.Nonzero),
		allowed_pods: p32(n.AllowedPods), pod_count: p32(n.PodCount), unschedulable: pu8(n.Unschedulable),
		n_label_cols: C.int32_t(n.NLabelCols), label_val: pu32(n.LabelVal), label_num: p64(n.LabelNum),
		label_num_ok: pu8(n.LabelNumOK), max_taints: C.int32_t(n.MaxTaints), taints: pu32(n.Taints),
		n_taint_vocab: C.int32_t(len(n.TaintEffect)), taint_effect: pu8(n.TaintEffect),
		max_images: C.int32_t(n.MaxImages), images: pu32(n.Images), n_images: C.int32_t(n.NImages),
	}
	x.nN = n.NNodes
	return x.check(C.ksg_load_nodes(x.c, &cn, topo))
}

// SetProfile installs the encoded scheduler profile (MultiPoint order,
// weights from getScorePluginWeight, plugin args).
func (x *Ctx) SetProfile(p *C.ksg_profile) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	return x.check(C.ksg_set_profile(x.c, p))
}

// LoadWorkload uploads encoded pods and their program pool.
func (x *Ctx) LoadWorkload(pods []C.ksg_pod, prog []int32) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	wl := C.ksg_workload{n_pods: C.int32_t(len(pods)), prog: p32(prog), prog_len: C.int64_t(len(prog))}
	if len(pods) > 0 {
		wl.pods = &pods[0]
	}
	return x.check(C.ksg_load_workload(x.c, &wl))
}

// PodEval is everything the wrapped plugins record for one pod, in SoA form.
// From EvalView the rows stay in the library's pinned block (ksg_eval_view):
// valid until the next evaluation on the context; from Eval they are copied
// into Go memory.
type PodEval struct {
	Selected, NFeasible int
	Status, ScoreSkip   uint32
	FStatus             []uint32 // [n_nodes]
	n, elem             int
	raw, norm           [NPlugins]unsafe.Pointer
	total               unsafe.Pointer
	keep                [][]int64 // Eval: the Go rows the pointers above refer to
	// the normalised rows the per-cycle kernel leaves to the caller
	// (ksg_eval_rows.norm_from_raw): derived from raw and normMax
	normFromRaw, normScored uint32
	normMax                 [NPlugins]int64
}

func (e *PodEval) at(p unsafe.Pointer, node int) int64 {
	if p == nil {
		return 0
	}
	switch e.elem {
	case 1:
		return int64(*(*uint8)(unsafe.Add(p, node)))
	case 2:
		return int64(*(*int16)(unsafe.Add(p, 2*node)))
	case 4:
		return int64(*(*int32)(unsafe.Add(p, 4*node)))
	}
	return *(*int64)(unsafe.Add(p, 8*node))
}

// Raw is plugin's Score() value at node (0 for a plugin the profile does not score).
func (e *PodEval) Raw(plugin, node int) int64 { return e.at(e.raw[plugin], node) }

// Norm is plugin's value after NormalizeScore at node.  TaintToleration and
// NodeAffinity on the node-local per-cycle path are DefaultNormalizeScore of
// the raw value with the device's maximum over the feasible nodes (reverse
// for TaintToleration), computed here: the kernel no longer stores them.
func (e *PodEval) Norm(plugin, node int) int64 {
	if e.normFromRaw>>uint(plugin)&1 == 0 {
		return e.at(e.norm[plugin], node)
	}
	if e.normScored>>uint(plugin)&1 == 0 || e.FStatus[node] != 0 {
		return 0
	}
	raw, mx := e.at(e.raw[plugin], node), e.normMax[plugin]
	if plugin == TaintToleration {
		if mx == 0 {
			return 100
		}
		return 100 - 100*raw/mx
	}
	if mx == 0 {
		return raw
	}
	return 100 * raw / mx
}

// Total is the weighted sum at node (0: not scored, or not materialised:
// the node-local per-cycle path leaves it out, the framework sums the
// weights itself).
func (e *PodEval) Total(node int) int64 { return e.at(e.total, node) }

// NumNodes is the number of node columns.
func (e *PodEval) NumNodes() int { return e.n }

// EvalView runs the full per-pod sweep (filters in profile order with
// first-rejection exit, raw scores, normalisation, weighted totals, selectHost)
// without changing node state, leaving the rows in library memory (no copy).
// One call per pod, at PreFilter time.
func (x *Ctx) EvalView(pod int) (*PodEval, error) {
	x.mu.Lock()
	defer x.mu.Unlock()
	var res C.ksg_result
	var rows C.ksg_eval_rows
	if err := x.check(C.ksg_eval_view(x.c, C.int32_t(pod), &res, &rows)); err != nil {
		return nil, err
	}
	e := &PodEval{n: int(rows.n_nodes), elem: int(rows.elem_bytes)}
	e.FStatus = unsafe.Slice((*uint32)(unsafe.Pointer(rows.fstatus)), e.n)
	for p := 0; p < NPlugins; p++ {
		e.raw[p], e.norm[p] = unsafe.Pointer(rows.raw[p]), unsafe.Pointer(rows.norm[p])
	}
	e.total = unsafe.Pointer(rows.total)
	e.normFromRaw, e.normScored = uint32(rows.norm_from_raw), uint32(rows.norm_scored)
	for p := 0; p < NPlugins; p++ {
		e.normMax[p] = int64(rows.norm_max[p])
	}
	e.Selected, e.NFeasible = int(res.selected), int(res.n_feasible)
	e.Status, e.ScoreSkip = uint32(res.status), uint32(res.score_skip)
	return e, nil
}

// Eval is EvalView with the rows copied into Go memory (they survive later
// evaluations).
func (x *Ctx) Eval(pod int) (*PodEval, error) {
	x.mu.Lock()
	defer x.mu.Unlock()
	n := x.nN
	fs, raw, norm, total := make([]uint32, n), make([]int64, NPlugins*n), make([]int64, NPlugins*n), make([]int64, n)
	var res C.ksg_result
	cap := C.ksg_capture{fstatus: pu32(fs), raw: p64(raw), norm: p64(norm), total: p64(total)}
	if err := x.check(C.ksg_eval(x.c, C.int32_t(pod), &res, &cap)); err != nil {
		return nil, err
	}
	e := &PodEval{FStatus: fs, n: n, elem: 8, keep: [][]int64{raw, norm, total}}
	for p := 0; p < NPlugins; p++ {
		e.raw[p], e.norm[p] = unsafe.Pointer(&raw[p*n]), unsafe.Pointer(&norm[p*n])
	}
	e.total = unsafe.Pointer(&total[0])
	e.Selected, e.NFeasible = int(res.selected), int(res.n_feasible)
	e.Status, e.ScoreSkip = uint32(res.status), uint32(res.score_skip)
	return e, nil
}

// Commit assumes pod onto node (Reserve).
func (x *Ctx) Commit(pod, node int) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	return x.check(C.ksg_commit(x.c, C.int32_t(pod), C.int32_t(node)))
}

// Uncommit deletes a preemption victim from the node state (ksg_uncommit,
// the inverse of Commit).
func (x *Ctx) Uncommit(pod, node int) error {
	x.mu.Lock()
	defer x.mu.Unlock()
	return x.check(C.ksg_uncommit(x.c, C.int32_t(pod), C.int32_t(node)))
}

// PreemptVictims runs DefaultPreemption's SelectVictimsOnNode for every
// candidate node at once (ksg_preempt_victims).  cand[k]'s potential victims
// are vic[off[k]:off[k+1]], most important first; fits[k] == 0 means the node
// cannot help, victim[i] == 1 means vic[i] stays evicted.
func (x *Ctx) PreemptVictims(pod int, cand, off, vic []int32) (fits []int32, victim []uint8, err error) {
	x.mu.Lock()
	defer x.mu.Unlock()
	if len(off) != len(cand)+1 {
		return nil, nil, fmt.Errorf("ksched: off needs len(cand)+1 entries")
	}
	fits = make([]int32, len(cand))
	victim = make([]uint8, len(vic))
	if len(cand) == 0 {
		return fits, victim, nil
	}
	err = x.check(C.ksg_preempt_victims(x.c, C.int32_t(pod), p32(cand), C.int32_t(len(cand)), p32(off),
		p32(vic), p32(fits), pu8(victim)))
	return fits, victim, err
}

// EvalSkipping evaluates loaded pod `pod` with the Filter plugins in the
// skip bit mask skipped (ksg_eval_skipping) and returns the filter status
// words: DefaultPreemption's node-static verdict (status 0 = every filter
// outside the mask passes the node).
func (x *Ctx) EvalSkipping(pod int, skip uint32) ([]uint32, error) {
	x.mu.Lock()
	defer x.mu.Unlock()
	n := x.nN
	fs, raw, norm, total := make([]uint32, n), make([]int64, NPlugins*n), make([]int64, NPlugins*n), make([]int64, n)
	var res C.ksg_result
	cap := C.ksg_capture{fstatus: pu32(fs), raw: p64(raw), norm: p64(norm), total: p64(total)}
	if err := x.check(C.ksg_eval_skipping(x.c, C.int32_t(pod), C.uint32_t(skip), &res, &cap)); err != nil {
		return nil, err
	}
	return fs, nil
}

// RunQueue schedules pods [first, first+count) on the device in queue order.
func (x *Ctx) RunQueue(first, count int) ([]int32, error) {
	x.mu.Lock()
	defer x.mu.Unlock()
	pl := make([]int32, count)
	if count == 0 {
		return pl, nil
	}
	return pl, x.check(C.ksg_run_queue(x.c, C.int32_t(first), C.int32_t(count), p32(pl), nil, nil))
}
