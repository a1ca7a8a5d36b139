// Snapshot encoder binding (include/ksched_snapshot.h): v1.Node / v1.Pod ->
// the flat C views the native encoder reads.  Every view lives in C memory
// (an arena freed after the call), so no Go pointer crosses into C (cgo
// pointer rules).  Source only: no Go toolchain in this image (DESIGN.md §1).
package ksched

/*
#include <stdlib.h>
#include "ksched_snapshot.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	storagev1 "k8s.io/api/storage/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/selection"
)

// framework.Code values returned by Status / PreFilter (include/ksched_snapshot.h).
const (
	CodeSuccess                      = int(C.KSG_CODE_SUCCESS)
	CodeUnschedulable                = int(C.KSG_CODE_UNSCHEDULABLE)
	CodeUnschedulableAndUnresolvable = int(C.KSG_CODE_UNSCHEDULABLE_AND_UNRESOLVABLE)
	CodeSkip                         = int(C.KSG_CODE_SKIP)
)

// arena owns the C memory of one call's views.
type arena struct{ ptrs []unsafe.Pointer }

func (a *arena) alloc(n int, size C.size_t) unsafe.Pointer {
	if n < 1 {
		n = 1
	}
	p := C.calloc(C.size_t(n), size)
	a.ptrs = append(a.ptrs, p)
	return p
}

func (a *arena) str(s string) *C.char {
	p := C.CString(s)
	a.ptrs = append(a.ptrs, unsafe.Pointer(p))
	return p
}

func (a *arena) free() {
	for _, p := range a.ptrs {
		C.free(p)
	}
	a.ptrs = nil
}

func (a *arena) strs(ss []string) (C.int32_t, **C.char) {
	arr := unsafe.Slice((**C.char)(a.alloc(len(ss)+1, C.size_t(unsafe.Sizeof((*C.char)(nil))))), len(ss)+1)
	for i, s := range ss {
		arr[i] = a.str(s)
	}
	return C.int32_t(len(ss)), &arr[0]
}

func (a *arena) pairs(m map[string]string) (C.int32_t, *C.ksg_str_pair) {
	arr := unsafe.Slice((*C.ksg_str_pair)(a.alloc(len(m)+1, C.sizeof_ksg_str_pair)), len(m)+1)
	i := 0
	for k, v := range m { // order is irrelevant: the encoder keys by name
		arr[i].key, arr[i].value = a.str(k), a.str(v)
		i++
	}
	return C.int32_t(len(m)), &arr[0]
}

// quantity: cpu in millicores (Quantity.MilliValue), the rest in base units.
func (a *arena) resources(rl v1.ResourceList) (C.int32_t, *C.ksg_quantity) {
	arr := unsafe.Slice((*C.ksg_quantity)(a.alloc(len(rl)+1, C.sizeof_ksg_quantity)), len(rl)+1)
	i := 0
	for name, q := range rl {
		arr[i].name = a.str(string(name))
		if name == v1.ResourceCPU {
			arr[i].value = C.int64_t(q.MilliValue())
		} else {
			arr[i].value = C.int64_t(q.Value())
		}
		i++
	}
	return C.int32_t(len(rl)), &arr[0]
}

func (a *arena) nodeReqs(rs []v1.NodeSelectorRequirement) (C.int32_t, *C.ksg_requirement_view) {
	arr := unsafe.Slice((*C.ksg_requirement_view)(a.alloc(len(rs)+1, C.sizeof_ksg_requirement_view)), len(rs)+1)
	for i, r := range rs {
		arr[i].key, arr[i].op = a.str(r.Key), a.str(string(r.Operator))
		arr[i].n_values, arr[i].values = a.strs(r.Values)
	}
	return C.int32_t(len(rs)), &arr[0]
}

func (a *arena) labelReqs(rs []metav1.LabelSelectorRequirement) (C.int32_t, *C.ksg_requirement_view) {
	arr := unsafe.Slice((*C.ksg_requirement_view)(a.alloc(len(rs)+1, C.sizeof_ksg_requirement_view)), len(rs)+1)
	for i, r := range rs {
		arr[i].key, arr[i].op = a.str(r.Key), a.str(string(r.Operator))
		arr[i].n_values, arr[i].values = a.strs(r.Values)
	}
	return C.int32_t(len(rs)), &arr[0]
}

func (a *arena) term(t v1.NodeSelectorTerm) C.ksg_node_selector_term_view {
	var v C.ksg_node_selector_term_view
	v.n_expr, v.expr = a.nodeReqs(t.MatchExpressions)
	v.n_fields, v.fields = a.nodeReqs(t.MatchFields)
	return v
}

func (a *arena) selector(ls *metav1.LabelSelector) C.ksg_label_selector_view {
	var v C.ksg_label_selector_view
	if ls == nil {
		return v // nil: labels.Nothing()
	}
	v.is_set = 1
	v.n_labels, v.match_labels = a.pairs(ls.MatchLabels)
	v.n_expr, v.expr = a.labelReqs(ls.MatchExpressions)
	return v
}

// selectorOf turns a labels.Selector (helper.DefaultSelector's result) back
// into matchExpressions; nil = no default constraints.
func (a *arena) selectorOf(sel labels.Selector) C.ksg_label_selector_view {
	var v C.ksg_label_selector_view
	if sel == nil {
		return v
	}
	reqs, _ := sel.Requirements()
	out := make([]metav1.LabelSelectorRequirement, 0, len(reqs))
	for _, r := range reqs {
		var op metav1.LabelSelectorOperator
		switch r.Operator() {
		case selection.In, selection.Equals, selection.DoubleEquals:
			op = metav1.LabelSelectorOpIn
		case selection.NotIn, selection.NotEquals:
			op = metav1.LabelSelectorOpNotIn
		case selection.Exists:
			op = metav1.LabelSelectorOpExists
		case selection.DoesNotExist:
			op = metav1.LabelSelectorOpDoesNotExist
		default:
			op = metav1.LabelSelectorOperator(r.Operator())
		}
		out = append(out, metav1.LabelSelectorRequirement{Key: r.Key(), Operator: op, Values: r.Values().List()})
	}
	return a.selector(&metav1.LabelSelector{MatchExpressions: out})
}

func (a *arena) affinity(ts []v1.PodAffinityTerm, ws []v1.WeightedPodAffinityTerm) (C.int32_t, *C.ksg_affinity_term_view) {
	n := len(ts) + len(ws)
	arr := unsafe.Slice((*C.ksg_affinity_term_view)(a.alloc(n+1, C.sizeof_ksg_affinity_term_view)), n+1)
	fill := func(i int, w int32, t v1.PodAffinityTerm) {
		arr[i].weight = C.int32_t(w)
		arr[i].selector = a.selector(t.LabelSelector)
		arr[i].topology_key = a.str(t.TopologyKey)
		arr[i].n_namespaces, arr[i].namespaces = a.strs(t.Namespaces)
		arr[i].namespace_selector = a.selector(t.NamespaceSelector)
	}
	for i, t := range ts {
		fill(i, 0, t)
	}
	for i, w := range ws {
		fill(len(ts)+i, w.Weight, w.PodAffinityTerm)
	}
	return C.int32_t(n), &arr[0]
}

func (a *arena) containers(cs []v1.Container, init bool) (C.int32_t, *C.ksg_container_view) {
	arr := unsafe.Slice((*C.ksg_container_view)(a.alloc(len(cs)+1, C.sizeof_ksg_container_view)), len(cs)+1)
	for i, c := range cs {
		arr[i].image = a.str(c.Image)
		arr[i].n_requests, arr[i].requests = a.resources(c.Resources.Requests)
		if init && c.RestartPolicy != nil && *c.RestartPolicy == v1.ContainerRestartPolicyAlways {
			arr[i].restartable = 1
		}
		hp := unsafe.Slice((*C.ksg_host_port_view)(a.alloc(len(c.Ports)+1, C.sizeof_ksg_host_port_view)), len(c.Ports)+1)
		n := 0
		for _, p := range c.Ports {
			if p.HostPort > 0 { // schedutil.GetHostPorts; "" ip / protocol sanitised natively
				hp[n].host_ip, hp[n].protocol = a.str(p.HostIP), a.str(string(p.Protocol))
				hp[n].host_port = C.int32_t(p.HostPort)
				n++
			}
		}
		arr[i].n_host_ports, arr[i].host_ports = C.int32_t(n), &hp[0]
	}
	return C.int32_t(len(cs)), &arr[0]
}

func (a *arena) node(n *v1.Node) *C.ksg_node_view {
	v := (*C.ksg_node_view)(a.alloc(1, C.sizeof_ksg_node_view))
	v.name = a.str(n.Name)
	v.n_labels, v.labels = a.pairs(n.Labels)
	ts := unsafe.Slice((*C.ksg_taint_view)(a.alloc(len(n.Spec.Taints)+1, C.sizeof_ksg_taint_view)), len(n.Spec.Taints)+1)
	for i, t := range n.Spec.Taints {
		ts[i].key, ts[i].value, ts[i].effect = a.str(t.Key), a.str(t.Value), a.str(string(t.Effect))
	}
	v.n_taints, v.taints = C.int32_t(len(n.Spec.Taints)), &ts[0]
	v.n_alloc, v.allocatable = a.resources(n.Status.Allocatable)
	if n.Spec.Unschedulable {
		v.unschedulable = 1
	}
	im := unsafe.Slice((*C.ksg_image_view)(a.alloc(len(n.Status.Images)+1, C.sizeof_ksg_image_view)), len(n.Status.Images)+1)
	for i, img := range n.Status.Images {
		im[i].n_names, im[i].names = a.strs(img.Names)
		im[i].size_bytes = C.int64_t(img.SizeBytes)
	}
	v.n_images, v.images = C.int32_t(len(n.Status.Images)), &im[0]
	return v
}

func (a *arena) pod(p *v1.Pod, defaultSel labels.Selector) *C.ksg_pod_view {
	v := (*C.ksg_pod_view)(a.alloc(1, C.sizeof_ksg_pod_view))
	v.namespace_, v.name = a.str(p.Namespace), a.str(p.Name)
	v.n_labels, v.labels = a.pairs(p.Labels)
	v.n_containers, v.containers = a.containers(p.Spec.Containers, false)
	v.n_init_containers, v.init_containers = a.containers(p.Spec.InitContainers, true)
	if p.Spec.Overhead != nil {
		v.has_overhead = 1
		v.n_overhead, v.overhead = a.resources(p.Spec.Overhead)
	}
	v.node_name = a.str(p.Spec.NodeName)
	if p.Spec.NodeSelector != nil {
		v.has_node_selector = 1
		v.n_node_selector, v.node_selector = a.pairs(p.Spec.NodeSelector)
	}
	if aff := p.Spec.Affinity; aff != nil {
		if na := aff.NodeAffinity; na != nil {
			if req := na.RequiredDuringSchedulingIgnoredDuringExecution; req != nil {
				v.has_na_required = 1
				terms := unsafe.Slice((*C.ksg_node_selector_term_view)(a.alloc(len(req.NodeSelectorTerms)+1,
					C.sizeof_ksg_node_selector_term_view)), len(req.NodeSelectorTerms)+1)
				for i, t := range req.NodeSelectorTerms {
					terms[i] = a.term(t)
				}
				v.n_na_required, v.na_required = C.int32_t(len(req.NodeSelectorTerms)), &terms[0]
			}
			if pref := na.PreferredDuringSchedulingIgnoredDuringExecution; pref != nil {
				v.has_na_preferred = 1
				pts := unsafe.Slice((*C.ksg_preferred_term_view)(a.alloc(len(pref)+1, C.sizeof_ksg_preferred_term_view)), len(pref)+1)
				for i, t := range pref {
					pts[i].weight = C.int32_t(t.Weight)
					pts[i].preference = a.term(t.Preference)
				}
				v.n_na_preferred, v.na_preferred = C.int32_t(len(pref)), &pts[0]
			}
		}
		if pa := aff.PodAffinity; pa != nil {
			v.n_pod_affinity_required, v.pod_affinity_required = a.affinity(pa.RequiredDuringSchedulingIgnoredDuringExecution, nil)
			v.n_pod_affinity_preferred, v.pod_affinity_preferred = a.affinity(nil, pa.PreferredDuringSchedulingIgnoredDuringExecution)
		}
		if pa := aff.PodAntiAffinity; pa != nil {
			v.n_pod_anti_affinity_required, v.pod_anti_affinity_required = a.affinity(pa.RequiredDuringSchedulingIgnoredDuringExecution, nil)
			v.n_pod_anti_affinity_preferred, v.pod_anti_affinity_preferred = a.affinity(nil, pa.PreferredDuringSchedulingIgnoredDuringExecution)
		}
	}
	tols := unsafe.Slice((*C.ksg_toleration_view)(a.alloc(len(p.Spec.Tolerations)+1, C.sizeof_ksg_toleration_view)), len(p.Spec.Tolerations)+1)
	for i, t := range p.Spec.Tolerations {
		tols[i].key, tols[i].op = a.str(t.Key), a.str(string(t.Operator))
		tols[i].value, tols[i].effect = a.str(t.Value), a.str(string(t.Effect))
	}
	v.n_tolerations, v.tolerations = C.int32_t(len(p.Spec.Tolerations)), &tols[0]
	v.n_spread, v.spread = a.spreads(p.Spec.TopologySpreadConstraints)
	v.default_spread_selector = a.selectorOf(defaultSel)
	if p.DeletionTimestamp != nil {
		v.terminating = 1
	}
	if p.Spec.Priority != nil {
		v.priority = C.int32_t(*p.Spec.Priority)
	}
	// the arena allocates max(len, 1) views: the slice covers exactly that
	nv := len(p.Spec.Volumes)
	if nv < 1 {
		nv = 1
	}
	vols := unsafe.Slice((*C.ksg_volume_view)(a.alloc(len(p.Spec.Volumes)+1, C.sizeof_ksg_volume_view)), nv)
	for i, vol := range p.Spec.Volumes {
		vols[i].name, vols[i].kind = a.str(vol.Name), a.str(volumeKind(&vol.VolumeSource))
		if vol.PersistentVolumeClaim != nil {
			vols[i].claim_name = a.str(vol.PersistentVolumeClaim.ClaimName)
		}
	}
	v.n_volumes, v.volumes = C.int32_t(len(p.Spec.Volumes)), &vols[0]
	return v
}

// volumeKind is the JSON key of the VolumeSource field that is set (the
// sources the volume plugins' PreFilter reacts to are named; any other one is
// "other", which they Skip).
func volumeKind(s *v1.VolumeSource) string {
	switch {
	case s.PersistentVolumeClaim != nil:
		return "persistentVolumeClaim"
	case s.Ephemeral != nil:
		return "ephemeral"
	case s.GCEPersistentDisk != nil:
		return "gcePersistentDisk"
	case s.AWSElasticBlockStore != nil:
		return "awsElasticBlockStore"
	case s.AzureDisk != nil:
		return "azureDisk"
	case s.AzureFile != nil:
		return "azureFile"
	case s.Cinder != nil:
		return "cinder"
	case s.VsphereVolume != nil:
		return "vsphereVolume"
	case s.PortworxVolume != nil:
		return "portworxVolume"
	case s.RBD != nil:
		return "rbd"
	case s.ISCSI != nil:
		return "iscsi"
	}
	return "other"
}

// Plugin is one configv1.Plugin (name, weight).
type Plugin struct {
	Name   string
	Weight int32
}

// PluginSet is one extension point's configv1.PluginSet after
// ConvertForSimulator (plugins.go:177-186): names may carry the Wrapped
// suffix; "*" in Disabled disables every MultiPoint default for the point.
type PluginSet struct {
	Enabled  []Plugin
	Disabled []string
}

// Extension points of ProfileArgs.Points (KSG_POINT_*).
const (
	PointPreFilter = int(C.KSG_POINT_PREFILTER)
	PointFilter    = int(C.KSG_POINT_FILTER)
	PointPreScore  = int(C.KSG_POINT_PRESCORE)
	PointScore     = int(C.KSG_POINT_SCORE)
	NPoints        = int(C.KSG_NPOINTS)
)

// ProfileArgs is profile 0 of the KubeSchedulerConfiguration as the
// evaluator models it: MultiPoint plugins in order with weights, the
// per-point sets, and the plugin args (filled by ApplyPluginArgs from the
// decoded runtime.Object each plugin factory receives).
type ProfileArgs struct {
	Plugins                               []Plugin
	Points                                [NPoints]PluginSet
	FitStrategy                           string           // LeastAllocated / MostAllocated / RequestedToCapacityRatio
	FitShape                              [][2]int32       // RequestedToCapacityRatio (utilization, score 0..10)
	FitResources, BAResources             map[string]int64 // name -> weight
	FitResourceOrder, BAResourceOrder     []string         // the args' list order
	FitIgnoredResources, FitIgnoredGroups []string
	HardPodAffinityWeight                 int32
	IgnorePreferredTermsOfExistingPods    bool
	PTSSystemDefaulted                    bool
	PTSDefaultConstraints                 []v1.TopologySpreadConstraint // defaultingType List
}

// spreads builds ksg_spread_view entries (a pod's constraints, or
// PodTopologySpreadArgs.defaultConstraints).
func (a *arena) spreads(tsc []v1.TopologySpreadConstraint) (C.int32_t, *C.ksg_spread_view) {
	nv := len(tsc)
	if nv < 1 {
		nv = 1
	}
	sp := unsafe.Slice((*C.ksg_spread_view)(a.alloc(len(tsc)+1, C.sizeof_ksg_spread_view)), nv)
	for i, c := range tsc {
		sp[i].max_skew = C.int32_t(c.MaxSkew)
		sp[i].topology_key = a.str(c.TopologyKey)
		sp[i].when_unsatisfiable = a.str(string(c.WhenUnsatisfiable))
		sp[i].selector = a.selector(c.LabelSelector)
		if c.MinDomains != nil {
			sp[i].min_domains = C.int32_t(*c.MinDomains)
		}
		if c.NodeAffinityPolicy != nil {
			sp[i].node_affinity_policy = a.str(string(*c.NodeAffinityPolicy))
		}
		if c.NodeTaintsPolicy != nil {
			sp[i].node_taints_policy = a.str(string(*c.NodeTaintsPolicy))
		}
		sp[i].n_match_label_keys, sp[i].match_label_keys = a.strs(c.MatchLabelKeys)
	}
	return C.int32_t(len(tsc)), &sp[0]
}

// Snapshot is one ksg_snapshot (not thread-safe; the caller serialises).
type Snapshot struct {
	s      *C.ksg_snapshot
	msgBuf []byte // Statuses' message texts, kept across calls (callers serialise, as the C snapshot requires)
}

func (x *Snapshot) check(rc C.int) error {
	if rc == 0 {
		return nil
	}
	return &Error{Code: int(rc), Msg: C.GoString(C.ksg_snapshot_error(x.s))}
}

// NewSnapshot creates an empty snapshot for the profile.
func NewSnapshot(p *ProfileArgs) (*Snapshot, error) {
	var a arena
	defer a.free()
	var pv C.ksg_profile_view
	pls := unsafe.Slice((*C.ksg_plugin_view)(a.alloc(len(p.Plugins)+1, C.sizeof_ksg_plugin_view)), len(p.Plugins)+1)
	for i, pl := range p.Plugins {
		pls[i].name, pls[i].weight = a.str(pl.Name), C.int32_t(pl.Weight)
	}
	pv.n_plugins, pv.plugins = C.int32_t(len(p.Plugins)), &pls[0]
	pv.fit_strategy = a.str(p.FitStrategy)
	list := func(order []string, w map[string]int64) (C.int32_t, *C.ksg_quantity) {
		arr := unsafe.Slice((*C.ksg_quantity)(a.alloc(len(order)+1, C.sizeof_ksg_quantity)), len(order)+1)
		for i, n := range order {
			arr[i].name, arr[i].value = a.str(n), C.int64_t(w[n])
		}
		return C.int32_t(len(order)), &arr[0]
	}
	pv.n_fit_resources, pv.fit_resources = list(p.FitResourceOrder, p.FitResources)
	pv.n_ba_resources, pv.ba_resources = list(p.BAResourceOrder, p.BAResources)
	pv.n_fit_ignored_resources, pv.fit_ignored_resources = a.strs(p.FitIgnoredResources)
	pv.n_fit_ignored_groups, pv.fit_ignored_groups = a.strs(p.FitIgnoredGroups)
	pv.hard_pod_affinity_weight = C.int32_t(p.HardPodAffinityWeight)
	if p.IgnorePreferredTermsOfExistingPods {
		pv.ignore_preferred_terms_of_existing_pods = 1
	}
	if p.PTSSystemDefaulted {
		pv.pts_system_defaulted = 1
	}
	n, nv := len(p.FitShape), len(p.FitShape)
	if nv < 1 {
		nv = 1
	}
	su := unsafe.Slice((*C.int32_t)(a.alloc(n, 4)), nv)
	ss := unsafe.Slice((*C.int32_t)(a.alloc(n, 4)), nv)
	for i, pt := range p.FitShape {
		su[i], ss[i] = C.int32_t(pt[0]), C.int32_t(pt[1])
	}
	pv.n_shape, pv.shape_utilization, pv.shape_score = C.int32_t(n), &su[0], &ss[0]
	pv.n_default_constraints, pv.default_constraints = a.spreads(p.PTSDefaultConstraints)
	for k := 0; k < NPoints; k++ {
		ps := p.Points[k]
		en := unsafe.Slice((*C.ksg_plugin_view)(a.alloc(len(ps.Enabled)+1, C.sizeof_ksg_plugin_view)), len(ps.Enabled)+1)
		for i, pl := range ps.Enabled {
			en[i].name, en[i].weight = a.str(pl.Name), C.int32_t(pl.Weight)
		}
		pv.points[k].n_enabled, pv.points[k].enabled = C.int32_t(len(ps.Enabled)), &en[0]
		pv.points[k].n_disabled, pv.points[k].disabled = a.strs(ps.Disabled)
	}
	x := &Snapshot{}
	if rc := C.ksg_snapshot_new(&pv, &x.s); rc != 0 {
		return nil, &Error{Code: int(rc), Msg: "ksg_snapshot_new: unsupported profile"}
	}
	return x, nil
}

// Free releases the snapshot.
func (x *Snapshot) Free() { C.ksg_snapshot_free(x.s); x.s = nil }

// AddNode appends a node (snapshot order = column order).
func (x *Snapshot) AddNode(n *v1.Node) (int, error) {
	var a arena
	defer a.free()
	var idx C.int32_t
	err := x.check(C.ksg_snapshot_add_node(x.s, a.node(n), &idx))
	return int(idx), err
}

// AddPod appends a pod; defaultSel = helper.DefaultSelector of the pod (nil: none).
func (x *Snapshot) AddPod(p *v1.Pod, defaultSel labels.Selector) (int, error) {
	var a arena
	defer a.free()
	var idx C.int32_t
	err := x.check(C.ksg_snapshot_add_pod(x.s, a.pod(p, defaultSel), &idx))
	return int(idx), err
}

// HintPod announces a pending pod (ksg_snapshot_hint_pod): its selectors and
// term templates join the encoding universe at the next Sync, so adding it
// when its cycle comes appends in place instead of re-encoding.
func (x *Snapshot) HintPod(p *v1.Pod, defaultSel labels.Selector) error {
	var a arena
	defer a.free()
	return x.check(C.ksg_snapshot_hint_pod(x.s, a.pod(p, defaultSel)))
}

// UnhintPod drops the hint of a pending pod deleted before it was added
// (ksg_snapshot_unhint_pod); adding a pod drops its hint by itself.
func (x *Snapshot) UnhintPod(namespace, name string) error {
	var a arena
	defer a.free()
	return x.check(C.ksg_snapshot_unhint_pod(x.s, a.str(namespace), a.str(name)))
}

// AddNamespace registers a namespace and its labels: namespaceSelector
// terms resolve against the namespaces added so far (re-resolved on change).
func (x *Snapshot) AddNamespace(ns *v1.Namespace) error {
	var a arena
	defer a.free()
	n, l := a.pairs(ns.Labels)
	return x.check(C.ksg_snapshot_add_namespace(x.s, a.str(ns.Name), n, l))
}

// pvSource is the JSON key of the PersistentVolumeSource that is set (the
// in-tree sources CSI migration translates are refused at encode).
func pvSource(s *v1.PersistentVolumeSource) string {
	switch {
	case s.CSI != nil:
		return "csi"
	case s.HostPath != nil:
		return "hostPath"
	case s.Local != nil:
		return "local"
	case s.NFS != nil:
		return "nfs"
	case s.GCEPersistentDisk != nil:
		return "gcePersistentDisk"
	case s.AWSElasticBlockStore != nil:
		return "awsElasticBlockStore"
	case s.AzureDisk != nil:
		return "azureDisk"
	case s.AzureFile != nil:
		return "azureFile"
	case s.Cinder != nil:
		return "cinder"
	case s.VsphereVolume != nil:
		return "vsphereVolume"
	case s.PortworxVolume != nil:
		return "portworxVolume"
	}
	return "other"
}

const annBetaStorageClass = "volume.beta.kubernetes.io/storage-class"

// AddPV adds or replaces a PersistentVolume (the volume plugins' PV lister;
// snapshot.go:34 pvs); the next encode is a full one.
func (x *Snapshot) AddPV(pv *v1.PersistentVolume) error {
	var a arena
	defer a.free()
	v := (*C.ksg_pv_view)(a.alloc(1, C.sizeof_ksg_pv_view))
	v.name = a.str(pv.Name)
	v.n_labels, v.labels = a.pairs(pv.Labels)
	sc := pv.Spec.StorageClassName // storagehelpers.GetPersistentVolumeClass
	if c, ok := pv.Annotations[annBetaStorageClass]; ok {
		sc = c
	}
	v.storage_class = a.str(sc)
	if r := pv.Spec.ClaimRef; r != nil {
		v.claim_namespace, v.claim_name = a.str(r.Namespace), a.str(r.Name)
	}
	v.source = a.str(pvSource(&pv.Spec.PersistentVolumeSource))
	if na := pv.Spec.NodeAffinity; na != nil && na.Required != nil {
		v.has_node_affinity = 1
		ts := na.Required.NodeSelectorTerms
		terms := unsafe.Slice((*C.ksg_node_selector_term_view)(a.alloc(len(ts)+1,
			C.sizeof_ksg_node_selector_term_view)), len(ts)+1)
		for i, t := range ts {
			terms[i] = a.term(t)
		}
		v.n_terms, v.terms = C.int32_t(len(ts)), &terms[0]
	}
	return x.check(C.ksg_snapshot_add_pv(x.s, v))
}

// AddPVC adds or replaces a PersistentVolumeClaim (snapshot.go:35 pvcs).
func (x *Snapshot) AddPVC(c *v1.PersistentVolumeClaim) error {
	var a arena
	defer a.free()
	v := (*C.ksg_pvc_view)(a.alloc(1, C.sizeof_ksg_pvc_view))
	v.namespace_, v.name = a.str(c.Namespace), a.str(c.Name)
	v.volume_name = a.str(c.Spec.VolumeName)
	sc := "" // storagehelpers.GetPersistentVolumeClaimClass
	if cl, ok := c.Annotations[annBetaStorageClass]; ok {
		sc = cl
	} else if c.Spec.StorageClassName != nil {
		sc = *c.Spec.StorageClassName
	}
	v.storage_class = a.str(sc)
	modes := make([]string, len(c.Spec.AccessModes))
	for i, m := range c.Spec.AccessModes {
		modes[i] = string(m)
	}
	v.n_access_modes, v.access_modes = a.strs(modes)
	v.n_annotations, v.annotations = a.pairs(c.Annotations)
	if c.DeletionTimestamp != nil {
		v.deleting = 1
	}
	return x.check(C.ksg_snapshot_add_pvc(x.s, v))
}

// ClearStorage drops every PV, claim and StorageClass
// (ksg_snapshot_clear_storage): a lister resync clears, then re-adds what the
// listers hold, so deleted objects leave the snapshot.
func (x *Snapshot) ClearStorage() error {
	return x.check(C.ksg_snapshot_clear_storage(x.s))
}

// AddStorageClass adds or replaces a StorageClass (snapshot.go:36).
func (x *Snapshot) AddStorageClass(sc *storagev1.StorageClass) error {
	var a arena
	defer a.free()
	v := (*C.ksg_storage_class_view)(a.alloc(1, C.sizeof_ksg_storage_class_view))
	v.name, v.provisioner = a.str(sc.Name), a.str(sc.Provisioner)
	mode := string(storagev1.VolumeBindingImmediate)
	if sc.VolumeBindingMode != nil {
		mode = string(*sc.VolumeBindingMode)
	}
	v.binding_mode = a.str(mode)
	terms := unsafe.Slice((*C.ksg_topology_term_view)(a.alloc(len(sc.AllowedTopologies)+1,
		C.sizeof_ksg_topology_term_view)), len(sc.AllowedTopologies)+1)
	for i, t := range sc.AllowedTopologies {
		reqs := unsafe.Slice((*C.ksg_topology_requirement_view)(a.alloc(len(t.MatchLabelExpressions)+1,
			C.sizeof_ksg_topology_requirement_view)), len(t.MatchLabelExpressions)+1)
		for k, r := range t.MatchLabelExpressions {
			reqs[k].key = a.str(r.Key)
			reqs[k].n_values, reqs[k].values = a.strs(r.Values)
		}
		terms[i].n_requirements, terms[i].requirements = C.int32_t(len(t.MatchLabelExpressions)), &reqs[0]
	}
	v.n_allowed_topologies, v.allowed_topologies = C.int32_t(len(sc.AllowedTopologies)), &terms[0]
	return x.check(C.ksg_snapshot_add_storage_class(x.s, v))
}

// Bind records a pod already running on a node (replayed at load).
func (x *Snapshot) Bind(pod, node int) error {
	return x.check(C.ksg_snapshot_bind(x.s, C.int32_t(pod), C.int32_t(node)))
}

// Load encodes and uploads everything into ctx (bindings replayed).
func (x *Snapshot) Load(ctx *Ctx) error {
	ctx.mu.Lock()
	defer ctx.mu.Unlock()
	if err := x.check(C.ksg_snapshot_load(x.s, ctx.c)); err != nil {
		return err
	}
	var n C.int32_t
	C.ksg_snapshot_counts(x.s, &n, nil, nil, nil)
	ctx.nN = int(n)
	return nil
}

// Sync brings ctx up to date after AddPod (append when the universe is unchanged).
func (x *Snapshot) Sync(ctx *Ctx) (appended bool, err error) {
	ctx.mu.Lock()
	defer ctx.mu.Unlock()
	var ap C.int32_t
	err = x.check(C.ksg_snapshot_sync(x.s, ctx.c, &ap))
	var n C.int32_t
	C.ksg_snapshot_counts(x.s, &n, nil, nil, nil)
	ctx.nN = int(n)
	return ap != 0, err
}

// Assume commits pod onto node (device state + binding record).
func (x *Snapshot) Assume(ctx *Ctx, pod, node int) error {
	ctx.mu.Lock()
	defer ctx.mu.Unlock()
	return x.check(C.ksg_snapshot_assume(x.s, ctx.c, C.int32_t(pod), C.int32_t(node)))
}

// Forget undoes an assume / binding (pod deleted, preemption victim).
func (x *Snapshot) Forget(ctx *Ctx, pod, node int) error {
	ctx.mu.Lock()
	defer ctx.mu.Unlock()
	return x.check(C.ksg_snapshot_forget(x.s, ctx.c, C.int32_t(pod), C.int32_t(node)))
}

// Status is the framework.Status (code, message) of a node's filter status word.
func (x *Snapshot) Status(pod int, word uint32, node int) (int, string, error) {
	var code, ln C.int32_t
	buf := (*C.char)(C.malloc(512))
	defer C.free(unsafe.Pointer(buf))
	if err := x.check(C.ksg_snapshot_status(x.s, C.int32_t(pod), C.uint32_t(word), C.int32_t(node), &code, buf, 512, &ln)); err != nil {
		return 0, "", err
	}
	if ln >= 512 {
		big := (*C.char)(C.malloc(C.size_t(ln) + 1))
		defer C.free(unsafe.Pointer(big))
		if err := x.check(C.ksg_snapshot_status(x.s, C.int32_t(pod), C.uint32_t(word), C.int32_t(node), &code, big, ln+1, &ln)); err != nil {
			return 0, "", err
		}
		return int(code), C.GoString(big), nil
	}
	return int(code), C.GoString(buf), nil
}

// StatusesKept is Statuses into arrays the C snapshot owns and keeps across
// calls (ksg_snapshot_statuses_kept): when the previous call rejected few
// nodes, only that call's and this call's rejected nodes are written.  codes
// and msg alias C memory: they are read-only and valid until the next
// StatusesKept call or Free, so a caller that keeps them past the cycle (in
// CycleState) copies them first.
func (x *Snapshot) StatusesKept(pod int, words []uint32) (codes, msg []int32, msgs []string, err error) {
	n := len(words)
	if n == 0 {
		return x.Statuses(pod, words)
	}
	if len(x.msgBuf) == 0 {
		x.msgBuf = make([]byte, 1<<16)
	}
	var nm C.int32_t
	var ln C.int64_t
	var pc, pm *C.int32_t
	call := func() error {
		return x.check(C.ksg_snapshot_statuses_kept(x.s, C.int32_t(pod), (*C.uint32_t)(unsafe.Pointer(&words[0])),
			C.int32_t(n), &pc, &pm, (*C.char)(unsafe.Pointer(&x.msgBuf[0])), C.int64_t(len(x.msgBuf)), &nm, &ln))
	}
	if err = call(); err != nil {
		return nil, nil, nil, err
	}
	if int64(ln) > int64(len(x.msgBuf)) { // the texts did not fit: once more (the arrays already hold this call's output)
		x.msgBuf = make([]byte, int64(ln)+1)
		if err = call(); err != nil {
			return nil, nil, nil, err
		}
	}
	codes = unsafe.Slice((*int32)(unsafe.Pointer(pc)), n)
	msg = unsafe.Slice((*int32)(unsafe.Pointer(pm)), n)
	raw := x.msgBuf[:ln]
	msgs = make([]string, 0, int(nm))
	start := 0
	for i := 0; i < len(raw) && len(msgs) < int(nm); i++ {
		if raw[i] == 0 {
			msgs = append(msgs, string(raw[start:i]))
			start = i + 1
		}
	}
	return codes, msg, msgs, nil
}

// Statuses decodes every node's Filter status word of a pod at once
// (ksg_snapshot_statuses): codes[n] (Code*), msg[n] = index into msgs, -1
// for success / not evaluated.  One C call writes straight into the result
// slices (plain int32 / uint32 memory, valid to pass for the call) and into
// the Snapshot's message buffer; a second call only when the texts outgrow it.
func (x *Snapshot) Statuses(pod int, words []uint32) (codes, msg []int32, msgs []string, err error) {
	n := len(words)
	codes = make([]int32, n, n+1) // capacity n+1: a valid first element even for n == 0
	msg = make([]int32, n, n+1)
	wp := words
	if n == 0 {
		wp = make([]uint32, 1)
	}
	if len(x.msgBuf) == 0 {
		x.msgBuf = make([]byte, 1<<16)
	}
	var nm C.int32_t
	var ln C.int64_t
	call := func() error {
		return x.check(C.ksg_snapshot_statuses(x.s, C.int32_t(pod), (*C.uint32_t)(unsafe.Pointer(&wp[0])), C.int32_t(n),
			(*C.int32_t)(unsafe.Pointer(&codes[:1][0])), (*C.int32_t)(unsafe.Pointer(&msg[:1][0])),
			(*C.char)(unsafe.Pointer(&x.msgBuf[0])), C.int64_t(len(x.msgBuf)), &nm, &ln))
	}
	if err = call(); err != nil {
		return nil, nil, nil, err
	}
	if int64(ln) > int64(len(x.msgBuf)) { // the texts did not fit: once more with a buffer that does
		x.msgBuf = make([]byte, int64(ln)+1)
		if err = call(); err != nil {
			return nil, nil, nil, err
		}
	}
	raw := x.msgBuf[:ln]
	msgs = make([]string, 0, int(nm))
	start := 0
	for i := 0; i < len(raw) && len(msgs) < int(nm); i++ {
		if raw[i] == 0 {
			msgs = append(msgs, string(raw[start:i]))
			start = i + 1
		}
	}
	return
}

// ProfileInfo is the profile as the framework and the Store see it
// (ksg_snapshot_profile_info): per-point run orders and the two weight maps.
type ProfileInfo struct {
	Order           [NPoints][]int
	StoreWeight     [NPlugins]int64 // getScorePluginWeight (plugins.go:289-304), 0 = absent
	SelectionWeight [NPlugins]int32
	NormalizeMask   uint32
}

// ProfileInfo returns the derived orders and weights.
func (x *Snapshot) ProfileInfo() (*ProfileInfo, error) {
	var ci C.ksg_profile_info
	if err := x.check(C.ksg_snapshot_profile_info(x.s, &ci)); err != nil {
		return nil, err
	}
	out := &ProfileInfo{NormalizeMask: uint32(ci.normalize_mask)}
	for k := 0; k < NPoints; k++ {
		for i := 0; i < int(ci.n_order[k]); i++ {
			out.Order[k] = append(out.Order[k], int(ci.order[k][i]))
		}
	}
	for i := 0; i < NPlugins; i++ {
		out.StoreWeight[i] = int64(ci.store_weight[i])
		out.SelectionWeight[i] = int32(ci.selection_weight[i])
	}
	return out, nil
}

// PreFilter is plugin's PreFilter code for the pod and, for NodeAffinity,
// the PreFilterResult node names (nil when it has none).
func (x *Snapshot) PreFilter(pod, plugin int, resultStatus uint32) (int, []string, error) {
	var code, has, n C.int32_t
	if err := x.check(C.ksg_snapshot_prefilter(x.s, C.int32_t(pod), C.int32_t(plugin), C.uint32_t(resultStatus), &code, &has, nil, 0, &n)); err != nil {
		return 0, nil, err
	}
	if has == 0 {
		return int(code), nil, nil
	}
	arr := (**C.char)(C.calloc(C.size_t(n)+1, C.size_t(unsafe.Sizeof((*C.char)(nil)))))
	defer C.free(unsafe.Pointer(arr))
	if err := x.check(C.ksg_snapshot_prefilter(x.s, C.int32_t(pod), C.int32_t(plugin), C.uint32_t(resultStatus), &code, &has, arr, n, &n)); err != nil {
		return 0, nil, err
	}
	names := make([]string, int(n))
	for i, p := range unsafe.Slice(arr, int(n)) {
		names[i] = C.GoString(p)
	}
	return int(code), names, nil
}

// NodeIndex returns the column of a node (-1: unknown).
// PreFilterMessage is the message of a PreFilter rejection of plugin
// (NodeAffinity's conflict, a volume plugin's claim / volume lookup; "" none).
func (x *Snapshot) PreFilterMessage(pod, plugin int) (string, error) {
	var n C.int32_t
	if err := x.check(C.ksg_snapshot_prefilter_message(x.s, C.int32_t(pod), C.int32_t(plugin), nil, 0, &n)); err != nil {
		return "", err
	}
	if n == 0 {
		return "", nil
	}
	buf := (*C.char)(C.malloc(C.size_t(n) + 1))
	defer C.free(unsafe.Pointer(buf))
	if err := x.check(C.ksg_snapshot_prefilter_message(x.s, C.int32_t(pod), C.int32_t(plugin), buf, n+1, &n)); err != nil {
		return "", err
	}
	return C.GoStringN(buf, n), nil
}

func (x *Snapshot) NodeIndex(name string) int {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var idx C.int32_t
	C.ksg_snapshot_node_index(x.s, cs, &idx)
	return int(idx)
}

var _ = fmt.Sprintf
