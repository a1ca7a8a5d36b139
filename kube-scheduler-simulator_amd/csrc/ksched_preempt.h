// DefaultPreemption dry run for preemptors whose PodTopologySpread or
// InterPodAffinity filter depends on the pods of the node (included by
// ksched.hip inside its anonymous namespace, after the queue kernels).
//
// Upstream SelectVictimsOnNode [k8s.io/kubernetes v1.32.5
// framework/preemption + plugins/defaultpreemption, not vendored] removes the
// lower-priority pods from a copy of the node, keeping the cloned PreFilter
// state in step through the plugins' RemovePod / AddPod extensions
// (podtopologyspread updateWithPod: the domain count of the node's value for
// every constraint whose selector matches the removed pod, when the node
// carries every constraint key and passes the inclusion policies, then the
// critical paths; interpodaffinity updateWithPod: the existing pods'
// anti-affinity counts of the removed pod's own terms, and the counts of the
// preemptor's affinity / anti-affinity terms that the removed pod matches),
// runs every filter, then reprieves the victims most important first.
//
// Here:
//   ksg_preempt_prepass   one workgroup: the preemptor's PreFilter state on the
//                         live node state (the queue kernel's pre-pass for the
//                         hard constraints and the required terms), plus, per
//                         hard constraint, how many domains hold the minimum
//                         and the smallest count above it;
//   ksg_preempt_topo      one lane per candidate node: the same removals and
//                         reprieves as the Fit-only kernel, with the domain
//                         counts of the candidate's own domains adjusted by
//                         the victims' selector / template memberships (their
//                         assume programs).  Only the candidate's domains
//                         change, so the new global minimum of a constraint is
//                         min(adjusted count, minimum over the other domains),
//                         the latter = the second smallest value when the
//                         candidate's domain alone holds the minimum.

constexpr int kPreMaxMAnti = 16;    // existing-pod anti-affinity templates per preemptor

struct PreemptTopo {
  long long m1[kMaxHard];     // minimum domain count (before the minDomains rule)
  long long m2[kMaxHard];     // smallest domain count above m1 (BIG: none)
  int32_t c1[kMaxHard];       // domains holding m1
  int32_t dom[kMaxHard];      // domains (eligible nodes' values)
  long long aff_total;
  int32_t ipa_skip_filter;
  int32_t ok;
  int32_t hist[KSG_HIST_MAX];
};

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void ksg_preempt_prepass(DevCluster c, DevState st, const ksg_pod* pods,
                                                             const int32_t* prog, const ksg_profile* profp, int pod,
                                                             PreemptTopo* out) {
  constexpr long long BIG = 0x7fffffffffffffffll;
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ TopoProg s_g;
  __shared__ TopoShared s_t;
  __shared__ int32_t s_hist[KSG_HIST_MAX];
  __shared__ unsigned long long s_m2[kMaxHard];
  __shared__ int32_t s_c1[kMaxHard];
  const int tid = threadIdx.x, lane = tid & 63;
  const int N = c.N;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(profp)[i_];
  stage_pod<BLOCK>(pods, prog, pod, &s_pod, s_blob);
  __syncthreads();
  const ksg_pod& p = s_pod;
  if (tid == 0) {
    const PodView v0 = make_view(c, s_prof, p, s_blob, prog, true);
    parse_topo(p, s_blob, v0.fskip, v0.smask, s_g);
    layout_slots(c, s_g, s_t);
    long long ma = 0;
    for (int i = 0; i < s_g.n_ma; i++) ma += st.tmpl_total[s_g.m_anti[i]];
    s_t.ipa_skip_filter = !s_g.ipa || (ma == 0 && s_g.n_aff == 0 && s_g.n_anti == 0);
    for (int i = 0; i < kMaxHard; i++) { s_t.hard_min[i] = BIG; s_t.hard_dom[i] = 0; s_m2[i] = BIG; s_c1[i] = 0; }
    s_t.aff_total = 0;
    // over the limits: nothing below touches the histograms (s_t.words may
    // exceed KSG_HIST_MAX then) and the host reports UNSUPPORTED
    s_t.ok = s_t.ok && s_g.n_ma <= kPreMaxMAnti;
    if (!s_t.ok) s_t.words = 0;
  }
  __syncthreads();
  for (int i = tid; i < s_t.words; i += BLOCK) s_hist[i] = 0;
  const PodView v = make_view(c, s_prof, p, s_blob, prog, true);
  const TopoProg& g = s_g;
  const int32_t* cnt = st.cnt;
  const bool ok = s_t.ok;
  __syncthreads();
  if (ok) {
    long long lmin[kMaxHard], laff = 0;
    int32_t ldom[kMaxHard];
    for (int i = 0; i < kMaxHard; i++) { lmin[i] = BIG; ldom[i] = 0; }
    for (int n = tid; n < N; n += BLOCK) {
      if (g.pts_filter && has_all(c, g.hard, g.n_hard, 7, n)) {
        for (int i = 0; i < g.n_hard; i++) {
          const int32_t* h = g.hard + 7 * i;
          if (!inclusion(c, v, h[5], h[6], n)) continue;
          const Slot& sl = s_t.hard[i];
          const int32_t x = cnt_at(cnt, N, sl.sel, n);
          if (sl.unique) {
            lmin[i] = min(lmin[i], (long long)x);
            ldom[i] += 1;
          } else {
            const uint32_t val = lab(c, sl.col, n);
            atomicAdd(&s_hist[sl.hist + val], x);
            atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
          }
        }
      }
      if (g.ipa) {
        if (g.n_aff > 0) {
          const int32_t x = cnt_at(cnt, N, g.sel_all, n);
          for (int i = 0; i < g.n_aff; i++) {
            const Slot& sl = s_t.aff[i];
            const uint32_t val = lab(c, sl.col, n);
            if (!val) continue;
            laff += x;
            if (!sl.unique) {
              atomicAdd(&s_hist[sl.hist + val], x);
              atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
            }
          }
        }
        for (int i = 0; i < g.n_anti; i++) {
          const Slot& sl = s_t.anti[i];
          const uint32_t val = lab(c, sl.col, n);
          if (!val || sl.unique) continue;
          atomicAdd(&s_hist[sl.hist + val], cnt_at(cnt, N, sl.sel, n));
          atomicOr((uint32_t*)&s_hist[sl.pres + (val >> 5)], 1u << (val & 31));
        }
      }
    }
    for (int i = 0; i < g.n_hard; i++) {
      const long long m = wave_min64(lmin[i]);
      const int32_t d = wave_sum32(ldom[i]);
      if (lane == 0 && s_t.hard[i].unique) {
        atomicMin((unsigned long long*)&s_t.hard_min[i], (unsigned long long)m);
        atomicAdd(&s_t.hard_dom[i], d);
      }
    }
    laff = wave_sum64(laff);
    if (lane == 0 && laff) atomicAdd((unsigned long long*)&s_t.aff_total, (unsigned long long)laff);
  }
  __syncthreads();
  if (ok) {   // minimum over the present domains of the non-unique hard slots
    for (int i = 0; i < g.n_hard; i++) {
      const Slot& sl = s_t.hard[i];
      if (sl.unique) continue;
      long long m = BIG;
      int32_t d = 0;
      for (int val = tid; val < sl.V; val += BLOCK)
        if (bit_get(s_hist, sl.pres, val)) { m = min(m, (long long)s_hist[sl.hist + val]); d += 1; }
      m = wave_min64(m);
      d = wave_sum32(d);
      if (lane == 0) {
        atomicMin((unsigned long long*)&s_t.hard_min[i], (unsigned long long)m);
        atomicAdd(&s_t.hard_dom[i], d);
      }
    }
  }
  __syncthreads();
  if (ok) {   // domains at the minimum and the smallest count above it
    for (int i = 0; i < g.n_hard; i++) {
      const Slot& sl = s_t.hard[i];
      const long long m1 = s_t.hard_min[i];
      int32_t c1 = 0;
      long long m2 = BIG;
      if (sl.unique) {
        const int32_t* h = g.hard + 7 * i;
        for (int n = tid; n < N; n += BLOCK) {
          if (!has_all(c, g.hard, g.n_hard, 7, n) || !inclusion(c, v, h[5], h[6], n)) continue;
          const long long x = cnt_at(cnt, N, sl.sel, n);
          if (x == m1) c1 += 1;
          else if (x > m1) m2 = min(m2, x);
        }
      } else {
        for (int val = tid; val < sl.V; val += BLOCK) {
          if (!bit_get(s_hist, sl.pres, val)) continue;
          const long long x = s_hist[sl.hist + val];
          if (x == m1) c1 += 1;
          else if (x > m1) m2 = min(m2, x);
        }
      }
      c1 = wave_sum32(c1);
      m2 = wave_min64(m2);
      if (lane == 0) {
        if (c1) atomicAdd(&s_c1[i], c1);
        atomicMin(&s_m2[i], (unsigned long long)m2);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < s_t.words; i += BLOCK) out->hist[i] = s_hist[i];
  if (tid == 0) {
    for (int i = 0; i < kMaxHard; i++) {
      out->m1[i] = s_t.hard_min[i];
      out->m2[i] = (long long)s_m2[i];
      out->c1[i] = s_c1[i];
      out->dom[i] = s_t.hard_dom[i];
    }
    out->aff_total = s_t.aff_total;
    out->ipa_skip_filter = s_t.ipa_skip_filter;
    out->ok = ok ? 1 : 0;
  }
}

// Membership of one pod (a victim) in the preemptor's counts, from its assume
// program: +sign per hard constraint / anti term selector it matches, on the
// affinity conjunction, and per existing anti-affinity template it owns.
struct PreDelta {
  int32_t pts[kMaxHard], anti[kMaxAnti], manti[kPreMaxMAnti];
  int32_t aff;
};

__device__ __forceinline__ void pre_delta(const TopoProg& g, const TopoShared& t, const int32_t* commit, int sign,
                                          PreDelta& d) {
  if (!commit) return;
  const int ns = commit[0];
  const int32_t* sels = commit + 1;
  for (int k = 0; k < ns; k++) {
    const int s = sels[k];
    for (int i = 0; i < g.n_hard; i++)
      if (t.hard[i].sel == s) d.pts[i] += sign;
    if (g.n_aff > 0 && g.sel_all == s) d.aff += sign;
    for (int i = 0; i < g.n_anti; i++)
      if (t.anti[i].sel == s) d.anti[i] += sign;
  }
  const int32_t* w = sels + ns;
  const int nt = *w++;
  for (int k = 0; k < nt; k++) {
    const int tm = w[2 * k];
    for (int i = 0; i < g.n_ma; i++)
      if (g.m_anti[i] == tm) d.manti[i] += sign;   // required anti-affinity: weight 1 in the table
  }
}

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_preempt_topo(DevCluster c, DevState st, const ksg_pod* pods,
                                                        const int32_t* prog, const ksg_profile* profp, int pod,
                                                        const PreemptTopo* topo, const int32_t* cand, int n_cand,
                                                        const int32_t* off, const int32_t* vic, int32_t* fits,
                                                        uint8_t* victim, int ports_on) {
  __shared__ int32_t s_blob[KSG_BLOB_MAX];
  __shared__ ksg_pod s_pod;
  __shared__ ksg_profile s_prof;
  __shared__ TopoProg s_g;
  __shared__ TopoShared s_t;
  const int tid = threadIdx.x;
  const int N = c.N;
  for (int i_ = tid; i_ < (int)(sizeof(ksg_profile) / 4); i_ += (int)blockDim.x)
    reinterpret_cast<int32_t*>(&s_prof)[i_] = reinterpret_cast<const int32_t*>(profp)[i_];
  stage_pod<256>(pods, prog, pod, &s_pod, s_blob);
  __syncthreads();
  const ksg_pod& p = s_pod;
  const ksg_profile& prof = s_prof;
  if (tid == 0) {
    const PodView v0 = make_view(c, prof, p, s_blob, prog, true);
    parse_topo(p, s_blob, v0.fskip, v0.smask, s_g);
    layout_slots(c, s_g, s_t);   // the prepass's layout: the histogram words index the same slots
  }
  __syncthreads();
  const int k = blockIdx.x * 256 + tid;
  if (k >= n_cand) return;
  if (!topo->ok) {   // the prepass refused the preemptor: PreDelta's arrays cannot hold its terms
    fits[k] = 0;
    for (int i = off[k]; i < off[k + 1]; i++) victim[i] = 0;
    return;
  }
  const PodView v = make_view(c, prof, p, s_blob, prog, true);
  const TopoProg& g = s_g;
  const TopoShared& t = s_t;
  bool fit_on = false, pts_on = false, ipa_on = false;
  for (int kf = 0; kf < prof.n_filter; kf++) {
    const int pl = prof.filter_order[kf];
    if ((v.fskip >> pl) & 1u) continue;
    fit_on |= pl == KSG_PL_NODE_RESOURCES_FIT;
    pts_on |= pl == KSG_PL_POD_TOPOLOGY_SPREAD;
    ipa_on |= pl == KSG_PL_INTER_POD_AFFINITY;
  }
  pts_on = pts_on && g.pts_filter;
  ipa_on = ipa_on && g.ipa && !topo->ipa_skip_filter;
  const int n = cand[k];
  NodeCols L;
  load_cols(c, st.requested, st.nonzero, st.pod_count, n, L);
  PreDelta d{};
  PrePorts pp;
  pp.init(ports_on ? prog + p.ports : nullptr, st.ports, N, n);
  const int b = off[k], e = off[k + 1];
  auto move = [&](int q, int sign) {
    const ksg_pod& w = pods[q];
    pp.move(w.ports >= 0 ? prog + w.ports : nullptr, sign);
#pragma unroll
    for (int r = 0; r < KSG_MAX_RES; r++)
      if (r < c.R) L.req[r] += sign * w.req[r];
    L.nz_cpu += sign * w.nz_cpu;
    L.nz_mem += sign * w.nz_mem;
    L.pod_count += sign;
    pre_delta(g, t, w.commit >= 0 ? prog + w.commit : nullptr, sign, d);
  };
  const bool all = pts_on && has_all(c, g.hard, g.n_hard, 7, n);
  auto passes = [&]() -> bool {
    if (!pp.ok()) return false;
    if (fit_on && fit_filter(c, p, L, prof.fit_ignored_res) != 0) return false;
    if (pts_on) {
      for (int i = 0; i < g.n_hard; i++) {
        const int32_t* h = g.hard + 7 * i;
        const uint32_t val = lab(c, h[0], n);
        if (!val) return false;
        const Slot& sl = t.hard[i];
        const bool incl = all && inclusion(c, v, h[5], h[6], n);
        const long long base = sl.unique ? (incl ? cnt_at(st.cnt, N, sl.sel, n) : 0) : hist_at(topo->hist, sl, val);
        const long long m1 = topo->m1[i];
        long long m = base, mn = m1;
        if (incl) {   // the candidate's domain is one of the counted domains: it moves
          m = base + d.pts[i];
          const long long others = (base == m1 && topo->c1[i] == 1) ? topo->m2[i] : m1;
          mn = m < others ? m : others;
        }
        if (topo->dom[i] < h[3]) mn = 0;   // minDomains
        if (m + h[4] - mn > h[2]) return false;
      }
    }
    if (ipa_on) {
      bool pods_exist = true;
      for (int i = 0; i < g.n_aff; i++) {
        const Slot& sl = t.aff[i];
        const uint32_t val = lab(c, sl.col, n);
        if (!val) return false;
        const long long m = (sl.unique ? cnt_at(st.cnt, N, g.sel_all, n) : hist_at(topo->hist, sl, val)) + d.aff;
        if (m <= 0) pods_exist = false;
      }
      const long long aff_total = topo->aff_total + (long long)d.aff * g.n_aff;
      if (!pods_exist && !(aff_total == 0 && g.n_aff > 0 && g.self_all)) return false;
      for (int i = 0; i < g.n_anti; i++) {
        const Slot& sl = t.anti[i];
        const uint32_t val = lab(c, sl.col, n);
        if (!val) continue;
        if ((sl.unique ? cnt_at(st.cnt, N, sl.sel, n) : hist_at(topo->hist, sl, val)) + d.anti[i] > 0) return false;
      }
      for (int i = 0; i < g.n_ma; i++) {
        const int tm = g.m_anti[i];
        const uint32_t val = lab(c, c.tmpl_col[tm], n);
        if (val && st.tab[c.tmpl_off[tm] + val] + d.manti[i] > 0) return false;
      }
    }
    return true;
  };
  for (int i = b; i < e; i++) move(vic[i], -1);
  const bool ok = passes();
  fits[k] = ok ? 1 : 0;
  for (int i = b; i < e; i++) {
    uint8_t out = 0;
    if (ok) {
      move(vic[i], +1);   // reprievePod
      if (!passes()) {
        move(vic[i], -1);
        out = 1;
      }
    }
    victim[i] = out;
  }
}
#endif  // KSG_PART
