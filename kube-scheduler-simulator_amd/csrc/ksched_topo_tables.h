// Domain tables maintained at assume time for the chip-wide topology path
// (ksched_topo_coop.h), included by ksched.hip inside its anonymous namespace.
//
// Upstream PodTopologySpread / InterPodAffinity PreFilter and PreScore count
// matching pods per topology domain by walking every pod of every node
// [upstream podtopologyspread/filtering.go calPreFilterState, scoring.go
// PreScore; interpodaffinity/filtering.go PreFilter].  The topology kernel's
// phase 1 folded the per-node selector counts cnt[s][n] into per-domain
// histograms for every pod (a node loop, a merge of G partial histograms and a
// grid barrier).  Here the domain counts are kept as state instead, updated
// O(1) per assume:
//
//   dom[(s, c)][v]  Σ cnt[s][n] over the nodes whose label column c (a
//                   non-unique topology key) has value v
//   tot[s]          Σ cnt[s][n] over every node
//   cc[s][k]        how many nodes have cnt[s][n] == k, for the selectors of
//                   hard constraints on a unique key (hostname): its minimum
//                   over the nodes is the smallest k with cc[s][k] > 0
//   pres[c]         the values of column c that some node has (static)
//
// They are exact for a pod whose constraints count over every node (default
// inclusion policies, every node carries the keys: col_missing),
// which then skips phase 1 and its barrier.  Assumes reach the tables one pod
// late (the lag lets the kernel run two grid barriers per pod; see
// ksched_topo_coop.h) and every reader adds the pending delta itself.

struct TopoTables {
  int32_t* dom;                // dom words
  int32_t* tot;                // [S]
  int32_t* cc;                 // cc words: [Kc] per registered selector
  const int32_t* pair_off;     // [S][L]: offset of (s, c)'s table in dom, -1 none
  const int32_t* cc_off;       // [S]: offset of s's count-of-counts in cc, -1 none
  uint32_t* pres;              // presence bitmaps
  const int32_t* pres_off;     // [L]: offset of c's bitmap in pres (words), -1 none
  int32_t* col_missing;        // [L]: 0 iff every node has label column c
  int32_t* col_empty;          // [L]: some node has the value "" (id 1)
  unsigned* invalid;           // set when a count or an assume did not fit: the tables go unused
  const int32_t* sp_off;       // [S + 1]: selector s's (column, dom offset) pairs are sp[2 * sp_off[s] ..]
  const int32_t* sp;
  const uint8_t* elig;         // [pods of the run]: the pod's constraints are all within the tables' scope
  const int4* fo;              // [pods of the run][kTopoFill]: per fill task (dom offset, presence offset,
                               // column, selector), in ksg_topo_coop's slot order
  int32_t first;               // the run's first pod (elig index 0)
  int32_t S, L, Kc;
};

// Whether every topology constraint of pod p counts over every node and has
// its table (the scope in which a pod reads the tables instead of running the
// pre-pass): default inclusion policies, every node carries the key (no node
// has "" for a unique soft key), each non-unique key's (selector, column)
// table and presence bitmap, each unique hard key's count-of-counts.  P: the
// program pool (absolute offsets).  Same program layout as parse_topo.
__device__ __forceinline__ bool tables_scope(const DevCluster& c, const TopoTables& tt, const ksg_pod& p,
                                             const int32_t* P, int base = 0) {
  auto pair = [&](int sel, int col) { return sel >= 0 ? tt.pair_off[(size_t)sel * tt.L + col] : -1; };
  auto all = [&](int col) { return tt.col_missing[col] == 0; };
  bool e = true;
  if (p.pts >= 0) {
    const int32_t* w = P + (p.pts - base);
    const int nh = w[0], ns = w[1];
    const int32_t* hard = w + 3;
    for (int i = 0; e && i < nh; i++) {
      const int32_t* h = hard + 7 * i;
      e = all(h[0]) && (!h[5] || p.na_req < 0) && !h[6] &&
          (c.col_unique[h[0]] ? h[1] >= 0 && tt.cc_off[h[1]] >= 0 : pair(h[1], h[0]) >= 0 && tt.pres_off[h[0]] >= 0);
    }
    const int32_t* soft = hard + 7 * nh;
    for (int i = 0; e && i < ns; i++) {
      const int32_t* sc = soft + 6 * i;
      e = all(sc[0]) && (!sc[3] || p.na_req < 0) && !sc[4] &&
          (sc[5] || (c.col_unique[sc[0]] ? tt.col_empty[sc[0]] == 0 : pair(sc[1], sc[0]) >= 0));
    }
  }
  if (p.ipa >= 0) {
    const int32_t* w = P + (p.ipa - base);
    const int na = w[0], sel_all = w[1];
    for (int i = 0; e && i < na; i++) {
      const int col = w[3 + i];
      e = c.col_unique[col] ? all(col) : pair(sel_all, col) >= 0 && tt.pres_off[col] >= 0;
    }
    w += 3 + na;
    const int nanti = *w++;
    for (int i = 0; e && i < nanti; i++) {
      const int col = w[2 * i];
      e = c.col_unique[col] || (pair(w[2 * i + 1], col) >= 0 && tt.pres_off[col] >= 0);
    }
    w += 2 * nanti;
    const int npref = *w++;
    for (int i = 0; e && i < npref; i++) {
      const int col = w[3 * i];
      e = c.col_unique[col] ? all(col) : pair(w[3 * i + 1], col) >= 0 && tt.pres_off[col] >= 0;
    }
  }
  return e;
}

constexpr int kTopoFill = 24;   // fill tasks per pod: kMaxHard + kMaxSoft + kMaxAff + kMaxAnti + kMaxPref

// tables_scope of pod p and its fill tasks: every non-unique slot's table
// offsets in the order the topology kernel lays its histograms out (hard,
// soft without a hostname key, affinity, anti-affinity, preferred), so the
// kernel's fill needs no dependent index load.  out: kTopoFill entries.
// prog + (offset - base) is the pod's program word at that offset (base 0:
// the pool; the pod's blob offset: its LDS copy).
__device__ __forceinline__ bool tables_fill(const DevCluster& c, const TopoTables& t, const ksg_pod& p,
                                            const int32_t* prog, int4* out, int base = 0) {
  const bool e = tables_scope(c, t, p, prog, base);
  int k = 0;
  auto task = [&](int sel, int col, bool pres) {
    if (k >= kTopoFill || col < 0 || col >= t.L || c.col_unique[col]) return;
    const int off = sel >= 0 && sel < t.S ? t.pair_off[(size_t)sel * t.L + col] : -1;
    out[k++] = make_int4(off, pres ? t.pres_off[col] : -1, col, sel);
  };
  if (e && p.pts >= 0) {
    const int32_t* w = prog + (p.pts - base);
    const int nh = w[0], ns = w[1];
    const int32_t* hard = w + 3;
    for (int j = 0; j < nh && j < kMaxHard; j++) task(hard[7 * j + 1], hard[7 * j], true);
    const int32_t* soft = hard + 7 * nh;
    for (int j = 0; j < ns && j < kMaxSoft; j++)
      if (!soft[6 * j + 5]) task(soft[6 * j + 1], soft[6 * j], false);
  }
  if (e && p.ipa >= 0) {
    const int32_t* w = prog + (p.ipa - base);
    const int na = w[0], sel_all = w[1];
    for (int j = 0; j < na && j < kMaxAff; j++) task(sel_all, w[3 + j], true);
    w += 3 + na;
    const int nanti = *w++;
    for (int j = 0; j < nanti && j < kMaxAnti; j++) task(w[2 * j + 1], w[2 * j], true);
    w += 2 * nanti;
    const int npref = *w++;
    for (int j = 0; j < npref && j < kMaxPref; j++) task(w[3 * j + 1], w[3 * j], true);
  }
  for (; k < kTopoFill; k++) out[k] = make_int4(-1, -1, -1, -1);
  return e;
}

// One lane per pod of the run: tables_fill into elig and fo (after ksg_topo_tables_init).
#ifndef KSG_PART
__global__ __launch_bounds__(64) void ksg_topo_tables_elig(DevCluster c, TopoTables t, const ksg_pod* pods,
                                                           const int32_t* prog, int count, uint8_t* elig,
                                                           int4* fo) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= count) return;
  elig[i] = tables_fill(c, t, pods[t.first + i], prog, fo + (size_t)i * kTopoFill) ? 1 : 0;
}
#endif  // KSG_PART

// One table-building task per workgroup (ksg_topo_tables_init).
struct TopoTableTask {
  int32_t kind;                // 0: dom[(s, c)] (+ pres[c] when first for c), 1: tot[s] + cc[s], 2: col_all /
                               // col_empty of column col
  int32_t sel, col, off, pres_off;
};

// Rebuild the tables from cnt and the labels: one workgroup per task, an LDS
// histogram over the task's values, one pass over the nodes.
constexpr int kTableLds = 8192;   // LDS words of a task's histogram (vocab / Kc bins)

#ifndef KSG_PART
__global__ __launch_bounds__(256) void ksg_topo_tables_init(DevCluster c, DevState st, TopoTables t,
                                                             const TopoTableTask* tasks) {
  __shared__ int32_t s_h[kTableLds];
  __shared__ int32_t s_tot;
  const TopoTableTask k = tasks[blockIdx.x];
  const int tid = threadIdx.x, N = c.N;
  if (k.kind == 2) {
    int missing = 0, empty = 0;
    for (int n = tid; n < N; n += 256) {
      const uint32_t v = lab(c, k.col, n);
      missing += v == 0;
      empty += v == 1;
    }
    missing = wave_sum32(missing);
    empty = wave_sum32(empty);
    if ((tid & 63) == 0) {
      if (missing) atomicAdd(&t.col_missing[k.col], 1);   // counts the waves that saw a missing label
      if (empty) atomicAdd(&t.col_empty[k.col], 1);
    }
    return;
  }
  const int bins = k.kind == 0 ? c.col_vocab[k.col] : t.Kc;
  for (int i = tid; i < bins && i < kTableLds; i += 256) s_h[i] = 0;
  if (tid == 0) s_tot = 0;
  __syncthreads();
  int32_t tot = 0;
  for (int n = tid; n < N; n += 256) {
    const int32_t x = st.cnt[(size_t)k.sel * N + n];
    if (k.kind == 0) {
      const uint32_t v = lab(c, k.col, n);
      if (v && x) atomicAdd(&s_h[v], x);
      if (k.pres_off >= 0 && v) atomicOr(&t.pres[k.pres_off + (v >> 5)], 1u << (v & 31));
    } else {
      tot += x;
      if (k.off >= 0) atomicAdd(&s_h[x < t.Kc - 1 ? x : t.Kc - 1], 1);
      if (k.off >= 0 && x >= t.Kc - 1) atomicOr(t.invalid, 1u);   // a count past the table
    }
  }
  tot = wave_sum32(tot);
  if ((tid & 63) == 0 && tot) atomicAdd(&s_tot, tot);
  __syncthreads();
  if (k.kind == 0) {
    for (int i = tid; i < bins; i += 256) t.dom[k.off + i] = s_h[i];
  } else {
    if (tid == 0) t.tot[k.sel] = s_tot;
    if (k.off >= 0)
      for (int i = tid; i < t.Kc; i += 256) t.cc[k.off + i] = s_h[i];
  }
}
#endif  // KSG_PART

// The pending effect of one assume on the tables and template tables, as every
// workgroup of the topology kernel knows it one pod late (the lag buffers).
constexpr int kLagSel = 8;    // matched selectors of the assumed pod that carry tables
constexpr int kLagTmpl = 8;   // templates the assumed pod owns

struct LagDelta {
  int node;                    // the assumed node (-1: nothing pending)
  int n_sel, n_tmpl;
  int sel[kLagSel];            // matched selectors (all of them when <= kLagSel)
  int old_cnt[kLagSel];        // cnt[sel][node] before the assume (the winner's published counts)
  int tidx[kLagTmpl];          // tab index tmpl_off[t] + label value (-1: the node lacks the key)
  int tw[kLagTmpl];            // the added weight (PREF: the term weight; else 1)
  int tt[kLagTmpl];            // the template
};
