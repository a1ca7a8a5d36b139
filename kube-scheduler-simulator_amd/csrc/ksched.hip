// libksched.so — MI355X (gfx950) Filter/Score evaluator behind the C ABI of
// include/ksched.h.
//
// Two execution schemes, both bit-exact with the sequential
// upstream cycle:
//
// 1. ksg_queue_kernel<BLOCK> — one workgroup per scheduling replica,
//    persistent over the pod queue.  Per pod: stage the pod into LDS; sweep A
//    (every lane walks nodes tid, tid+BLOCK, ...: filters in profile order with
//    first-rejection exit, raw scores); block reduction (feasible count, first
//    feasible node, normalisation maxima); sweep B (normalise, weight,
//    packed-key argmax = selectHost with lowest-index tie-break); one lane
//    assumes the pod.  Used for replica sweeps (config 4: one CU per
//    replica, no inter-workgroup traffic), for capture (annotation) runs and
//    for ksg_eval.
//
// 2. Batched speculate-and-repair, for a single replica's placement-only queue
//    when every enabled plugin is node-local (Fit, BalancedAllocation,
//    TaintToleration, NodeAffinity, ImageLocality, NodeUnschedulable,
//    NodeName): assuming a pod changes the columns of exactly one node, so
//    pod j of a batch sees the batch-start state everywhere except at the
//    <= j nodes chosen earlier in the batch.
//      ksg_batch_phase1  grid (node tiles, B pods): every (pod, node) of the
//                        batch against the batch-start state, packed into one
//                        8-byte record; per-pod normalisation maxima by atomics.
//      ksg_batch_phase2  one workgroup walks the batch in order: re-evaluates
//                        only the changed nodes against the live state, scans
//                        the records of the others, normalises with the live
//                        maxima (a second scan only if a max holder dropped
//                        out), selects and assumes.
//    Only the changed nodes are ever recomputed, so the result is the
//    sequential result exactly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <array>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "ksched_kernels.h"

#include "ksched_dev.h"
#include "ksched_json_host.h"

using namespace ksk;

#include "ksched_parts.h"

// ============================================================================
// Host side
// ============================================================================
struct ksg_ctx {
  int device = 0;
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_ms = 0;
  int last_path = 0;   // 1 = queue kernel, 2 = batched, 3 = replica sweep, 4 = chip-wide topology
  bool last_window = false;   // path 4 ran the speculative topology queue (ksched_topo_win.h)
  ksg_profile prof{};
  bool have_prof = false, have_nodes = false, have_wl = false;
  // cluster
  DevCluster c{};
  std::vector<void*> allocs;
  int32_t n_pods = 0;
  ksg_pod* d_pods = nullptr;
  int32_t* d_prog = nullptr;
  std::vector<ksg_pod> h_pods;
  std::vector<int32_t> h_na_pref_sum;   // per pod Σ preferred node-affinity weights
  std::vector<int32_t> h_prog;
  size_t pod_cap = 0, prog_cap = 0;   // device capacity of d_pods / d_prog (ksg_append_pods grows them)
  int64_t prog_used = 0;              // end of the last program word a loaded pod uses
  std::vector<int32_t> h_col_vocab;
  std::vector<uint8_t> h_col_unique;
  int32_t max_blob = 0;
  // state (replica 0 = the ctx's own state)
  DevState st{};
  size_t tab_words = 0;
  // load-time snapshot for ksg_reset_state
  int64_t* d_req0 = nullptr;
  int64_t* d_nz0 = nullptr;
  int32_t* d_pc0 = nullptr;
  // batched-path buffers (lazily allocated)
  uint64_t* d_rec = nullptr;
  int32_t* d_img = nullptr;
  int32_t* d_stat = nullptr;
  int32_t* d_pmax = nullptr;
  P1Stats* d_p1 = nullptr;
  uint64_t* d_top = nullptr;
  // pipelined path (two buffer sets by batch parity, a second stream for
  // phase 1 + top-k, the carried changed set)
  uint64_t* d_prec[2] = {nullptr, nullptr};
  int32_t* d_pimg[2] = {nullptr, nullptr};
  int32_t* d_pstat[2] = {nullptr, nullptr};
  int32_t* d_ppmax[2] = {nullptr, nullptr};
  P1Stats* d_pp1[2] = {nullptr, nullptr};
  uint64_t* d_ptop[2] = {nullptr, nullptr};
  int32_t* d_carry = nullptr;          // [2][KSG_BATCH_MAX] slot node lists, then [2] counts
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_tk[2] = {nullptr, nullptr}, ev_p2[2] = {nullptr, nullptr};
  int pipe_window = 1;                 // env KSG_PIPE_WINDOW=0: no overlap, no carried set
  // DefaultPreemption dry-run scratch (grow-only)
  int32_t* d_pre = nullptr;
  size_t pre_words = 0;
  PreemptTopo* d_pretopo = nullptr;    // topology dry run (ksched_preempt.h)
  ksg_profile* d_preprof = nullptr;
  // chip-wide topology path buffers (lazily allocated)
  CoopAcc* d_coop_acc = nullptr;
  unsigned* d_coop_flags = nullptr;   // [4] timeout, [6] the one-pod completion counter
  unsigned* d_coop_wgflags = nullptr; // [256][32] per-workgroup barrier flags
  int coop_pmode = 0;                 // env KSG_COOP_PMODE: 0 merge with atomics (33.3 k vs 32.1 k pods/s on
                                      // config 3), 1 every workgroup folds every partial slot
  CoopPart* d_coop_parts = nullptr;   // [256] per-workgroup partials
  int32_t* d_coop_phist = nullptr;    // [256][kCoopPHist] per-workgroup partial histograms
  uint64_t* d_coop_srec = nullptr;    // [kCoopBatch][N] static records of the current batch
  int coop_gmax = 0;                  // co-resident workgroups of ksg_topo_coop
  bool topo_coop = true;              // env KSG_TOPO_COOP=0 disables
  bool coop_tables = true;            // env KSG_COOP_TABLES=0: every pod runs phase 1 (no maintained tables)
  // a deferred assume (ksg_commit): applied by the next per-cycle kernel, or
  // launched by flush_commit before anything else reads the node state
  bool defer_commit = true;           // env KSG_DEFER_COMMIT=0 disables
  int32_t pc_pod = -1, pc_node = -1;
  int32_t* d_coop_notables = nullptr; // a zeroed word set standing for "no tables"
  // the chip-wide topology path's launch setup, kept across calls: the group
  // shape for cfg_N nodes, the barrier flag generation (no flag reset per
  // launch) and whether the flags / atomics sets / timeout word need a reset
  // (after an allocation or a failed launch; a completed launch leaves them clean)
  int coop_cfg_N = -1, coop_kn = 1, coop_G = 1;
  bool coop_ll = false;
  unsigned coop_gen = 0;
  bool coop_dirty = true;
  bool topo_eval_coop = false;        // the one-pod evaluation launches cooperatively (after a plain launch's
                                      // workgroups were not all resident)
  // Queue runs of the chip-wide topology path and the multi-workgroup replica
  // sweep: a plain launch of G workgroups within the occupancy API's
  // residency (checked before the launch), their barriers bounded by a
  // timeout.  env KSG_COOP_LAUNCH=1, or a barrier timeout, switches to
  // hipLaunchCooperativeKernel (a process that made cooperative launches
  // faulted in libamdhip64's exit-time teardown under rocprofv3).
  bool coop_launch = false;
  // the speculative topology queue (ksched_topo_win.h; env KSG_TOPO_WINDOW=0
  // disables): one device block for the rows' outputs, flags and partials
  bool topo_window = true;
  char* d_win = nullptr;
  size_t win_bytes = 0;
  int win_kmax = kWinMax;              // env KSG_TOPO_WINDOW_K: pods per window (1 .. kWinMax)
  unsigned long long win_stats[3] = {0, 0, 0};   // the last run: windows, pods decided, windows cut short
  int32_t* d_tables = nullptr;        // the maintained domain tables and their index (ksched_topo_tables.h)
  size_t tables_words = 0;
  // The per-cycle tables (ksg_eval of topology pods): the whole selector
  // universe's tables, built once, kept exact by ksg_commit's kernel,
  // invalidated by anything else that moves the counts (queue runs, reset,
  // reload, bulk bindings).  env KSG_PC_TABLES=0: the pre-pass every call.
  int32_t* d_pct = nullptr;
  size_t pct_words = 0;
  TopoTables pct{};
  bool pct_valid = false;
  bool pc_tables = true;
  unsigned* sweep_timeout = nullptr;  // the last replica sweep's group-barrier timeout word (S > 1)
  int force_path = 0;  // env KSG_FORCE_PATH: 1 queue kernel, 2 batched, 3 int64 sweep state
  bool last_narrow = false;   // the last replica sweep ran on the narrow records
  bool last_n32 = false;      // the last batched run's slot walk ran the 32-bit instances
  bool last_spec = false;     // ... the speculate-and-verify walk
  bool last_mw = false;       // ... in its wide-memory instance
  bool spec_persist = true;   // env KSG_SPEC_PERSIST=0: one spec-walk launch per batch (else one for the run)
  bool last_persist = false;  // the last batched run took the persistent walk (its state saved first)
  unsigned* h_p2done = nullptr;   // the persistent walk's batches-walked counter (pinned, mapped)
  unsigned* d_p2done = nullptr;
  int32_t* d_btab = nullptr;      // its batch table ([batch][6]; grown, freed with the context)
  size_t btab_cap = 0;
  std::vector<int32_t> h_btab;
  bool pipe_overlap = true;   // env KSG_PIPE_OVERLAP=0: the window pipeline on one stream (same arithmetic;
                              // for counter passes, which serialise kernels: a walk polling for the
                              // other stream's top-k would wait out its poll bound)
  uint64_t* d_prect[2] = {nullptr, nullptr};   // the spec walk: node-major record copies, per window parity
  int32_t* d_pimgt[2] = {nullptr, nullptr};    // ... and weight x ImageLocality
  unsigned* d_flag = nullptr; // range-check flag (ksg_range32)
  // env KSG_BATCH_MODE: 2 "slot" (one launch chain per batch), 4 "window" (the
  // slot walk in the two-stream pipeline), 6 "spec" (default: the
  // speculate-and-verify walk in the pipeline, the window slot walk outside
  // its scope).  Round 6 retired "scan", "topset" and "tcol" (never faster
  // than the window walk; the spec walk superseded them).
  // (default: the speculate-and-verify walk where the N32 check and spec_candidate pass,
  // else the window slot walk; both with the next batch's phase 1 + top-k overlapped
  // through the two-batch window)
  int batch_mode = 6;
  int slot_block = 64;   // env KSG_SLOT_BLOCK: pods per batch of the unwindowed slot walk: 64 or 128 (the window walk
                         // runs 64-pod batches, 416 k vs 408 k pods/s at 128, profiles/r2/phase2_window_blocks.log)
  // per-kernel timing (ksg_set_timing): one event before the first and after
  // every launch of a run, on the launch stream
  bool timing = false;
  std::vector<hipEvent_t> tev;
  int tev_used = 0;
  std::vector<std::pair<int, double>> tlaunch;   // (kernel kind, algorithmic units)
  double kstat_ms[KSG_NKERNELS] = {};
  double kstat_units[KSG_NKERNELS] = {};
  int32_t kstat_calls[KSG_NKERNELS] = {};
  unsigned long long* d_stamps = nullptr;   // KSG_STAMPS diagnostic build only
  // per-cycle evaluation (eval_fast): one grow-only device block and its
  // pinned host mirror, reused by every ksg_eval / ksg_eval_pod call
  char* d_ev = nullptr;
  size_t ev_bytes = 0;
  char* h_ev = nullptr;                     // hipHostMalloc'd, freed by ksg_close
  size_t h_ev_bytes = 0;
  char* d_hev = nullptr;                    // h_ev's device address (the kernel writes the results there)
  unsigned* pipe_tk = nullptr;              // the last run_pipe's top-k hand-off words (checked after the run)
  std::vector<uint32_t> view_fs;            // ksg_eval_view of a pod off the per-cycle path: library-owned rows
  std::vector<int64_t> view_rows;
  unsigned ev_seq = 0;                      // the per-cycle completion flag's last value
  bool ev_clean = false;                    // the arrival counter is zero
  ksg_profile* d_ev_prof = nullptr;
  int32_t* d_ev_pl = nullptr;               // eval_topo_fast's placement word
  // the device annotation serialiser (ksg_annotator_attach / ksg_run_queue_json)
  char* d_json_tab = nullptr;               // the uploaded tables (one block)
  JsonTables json_t{};
  int json_N = -1;                          // node count the tables were built for (-1: none attached)
  int json_T = 0;
  int64_t json_w[KSG_NPLUGINS] = {};
  uint32_t json_norm = 0;
  char* d_json_scratch = nullptr;           // per-lane counts, totals, offsets (grown only)
  size_t json_scratch_bytes = 0;
  char* d_json_arena = nullptr;             // a chunk's placements, results and capture arrays (grown only):
  size_t json_arena_bytes = 0;              // no hipFree (a device-wide wait) between chunks
  // three slots rotate: chunk i is read by the caller while chunk i + 1 is
  // copied back and chunk i + 2 is computed (ksg_run_queue_json_async)
  static constexpr int kJsonSlots = 3;
  char* d_json_out[kJsonSlots] = {};        // a chunk's values on the device
  size_t json_out_cap[kJsonSlots] = {};
  char* h_json[kJsonSlots] = {};            // ... and in pinned host memory
  size_t h_json_cap[kJsonSlots] = {};
  std::vector<int64_t> json_off[kJsonSlots];   // [3 * count + 1]
  uint32_t* d_json_err = nullptr;           // [kJsonSlots] error words
  uint32_t* h_json_err = nullptr;           // ... pinned copies
  hipEvent_t json_copied[kJsonSlots] = {};  // the slot's copy-back done
  hipEvent_t json_written = nullptr;
  hipStream_t json_stream = nullptr;        // the copies back
  bool json_busy[kJsonSlots] = {};
  int json_next = 0;
  int json_last = -1;                       // the slot the last ksg_run_queue_json_async filled
  bool json_want = false;                   // run_internal: serialise the capture on the device
  char* h_evt = nullptr;                    // eval_topo_fast's pinned block (its own: eval_fast polls words
  size_t h_evt_bytes = 0;                   // that topology rows would otherwise overwrite)
  char* d_hevt = nullptr;
  bool ev_prof_dirty = true;
  bool eval_fast = true;                    // env KSG_EVAL_FAST=0: ksg_eval takes the queue kernel
  int inject_walk_err = 0;                  // env KSG_TEST_INJECT_WALK_ERR=1 (tests: the walk's guard reaches the host)
  // env KSG_TEST_INJECT_TIMEOUT (tests): a mask of grid-barrier launches whose
  // next plain launch starts with its sticky timeout word set, so its barriers
  // give up as if a workgroup were not resident (partial commits included):
  // 1 the topology queue, 2 the one-pod topology evaluation, 4 the replica
  // sweep (S > 1), 8 the per-cycle launch.  Each bit is consumed by its
  // launch.
  int inject_timeout = 0;
  int32_t recoveries = 0;                   // grid-barrier timeouts recovered by a cooperative relaunch
  char* d_state_bak = nullptr;              // the node state before a plain topology queue launch (its
  size_t state_bak_bytes = 0;               // timeout restores it and relaunches cooperatively)
  CycArgs cyc_args{};                       // ksg_eval_cycle's launch arguments, rebuilt in place per call
  unsigned cyc_last_G = 0;                  // the grid of the last per-cycle call (its counter counts multiples of it)
  // the persistent per-cycle server (ksched_cycle.h ksg_cycle_server; the default since round 6,
  // KSG_CYCLE_SERVER=0: one launch per cycle)
  bool srv_mode = true;
  bool srv_running = false;
  int srv_kn = 0;
  unsigned srv_G = 0;
  bool srv_img = false, srv_sys = false;
  CycStatic srv_static{};
  SrvMailbox* h_mb = nullptr;               // the mailbox as the host writes it: fine-grained device memory the
                                            // CPU maps through the BAR (mb_device), else pinned host memory
  bool mb_device = false;                   // the mailbox is device memory: every workgroup polls it directly
  void* mb_alloc = nullptr;                 // (its allocation, freed at close)
  char* d_srv = nullptr;                    // the server's device relay of the call (dalloc: freed with the context)
  const SrvMailbox* d_mb = nullptr;
  std::chrono::steady_clock::time_point srv_last{};
  int cycle_kn = 1;                         // env KSG_CYCLE_KN (1/2/4): the smallest nodes-per-lane tried (tests)
  bool cycle_sys = true;                    // system-scope host stores + a vmcnt wait (no L2 write-back); env
                                            // KSG_CYCLE_SYS=0: plain stores + __threadfence_system (round 4)
  bool cycle_coop = false;                  // per-cycle launch: plain (G within the occupancy API's residency,
                                            // ~7 us less host time); cooperative after an exchange timeout,
                                            // or always with env KSG_CYCLE_COOP=1
  int cycle_cap[3] = {0, 0, 0};             // co-resident ksg_eval_cycle workgroups per KN = 1, 2, 4 (0 = not queried)
  // pinned staging of ksg_append_pods (the per-cycle append needs no host wait)
  char* h_stage = nullptr;
  size_t h_stage_bytes = 0;
  const char* d_stage = nullptr;            // h_stage's device address (fine-grained: no stale GPU cache lines)
  // a staged append not yet copied to d_pods / d_prog: the next ksg_eval of
  // that pod reads it from the staging buffer and copies it on the device
  // (no copy launches in the cycle); any other call copies it first
  bool stage_pending = false;
  int32_t stage_first = 0, stage_n = 0;
  int64_t stage_base = 0, stage_len = 0;
  hipEvent_t ev_stage = nullptr;            // the last staged copy is done when this fires
};

namespace {

int fail(ksg_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

#define HIPC(ctx, expr)                                                                     \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(ctx, KSG_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));    \
  } while (0)

// A kernel's dynamic-LDS budget attribute, set once per (device, kernel,
// budget): the attribute is per device, and contexts on several devices (or
// threads) may open in one process.
int func_lds_attr(ksg_ctx* ctx, const void* f, size_t bytes) {
  static std::mutex mu;
  static std::set<std::tuple<int, const void*, size_t>> done;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_tuple(ctx->device, f, bytes);
  if (done.count(key)) return KSG_OK;
  HIPC(ctx, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  done.insert(key);
  return KSG_OK;
}

template <typename T>
int dalloc(ksg_ctx* ctx, T** p, size_t count) {
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  hipError_t e = hipMalloc((void**)p, bytes);
  if (e != hipSuccess) return fail(ctx, KSG_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  ctx->allocs.push_back(*p);
  return KSG_OK;
}

template <typename T>
int upload(ksg_ctx* ctx, T** p, const T* src, size_t count) {
  int rc = dalloc(ctx, p, count);
  if (rc) return rc;
  if (count) HIPC(ctx, hipMemcpyAsync(*p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  return KSG_OK;
}

template <typename T>
int upc(ksg_ctx* ctx, const T*& field, const T* src, size_t count) {
  T* p = nullptr;
  int rc = upload(ctx, &p, src, count);
  field = p;
  return rc;
}

void free_all(ksg_ctx* ctx) {
  ctx->json_N = -1;   // the serialiser's tables name the old nodes
  for (void* p : ctx->allocs) (void)hipFree(p);
  ctx->allocs.clear();
  ctx->stage_pending = false;   // its destination arrays are gone
  ctx->d_pods = nullptr;
  ctx->d_prog = nullptr;
  ctx->pod_cap = ctx->prog_cap = 0;
  ctx->d_pre = nullptr;
  ctx->d_pretopo = nullptr;
  ctx->d_flag = nullptr;
  ctx->d_preprof = nullptr;
  ctx->pre_words = 0;
  ctx->d_rec = nullptr;
  ctx->d_img = nullptr;
  ctx->d_stat = nullptr;
  ctx->d_prect[0] = ctx->d_prect[1] = nullptr;
  ctx->d_pimgt[0] = ctx->d_pimgt[1] = nullptr;
  ctx->d_pmax = nullptr;
  ctx->d_p1 = nullptr;
  ctx->d_top = nullptr;
  for (int q = 0; q < 2; q++) {
    ctx->d_prec[q] = nullptr;
    ctx->d_pimg[q] = nullptr;
    ctx->d_pstat[q] = nullptr;
    ctx->d_ppmax[q] = nullptr;
    ctx->d_pp1[q] = nullptr;
    ctx->d_ptop[q] = nullptr;
  }
  ctx->d_carry = nullptr;
  ctx->d_stamps = nullptr;
  ctx->d_coop_acc = nullptr;
  ctx->d_coop_flags = nullptr;
  ctx->d_coop_wgflags = nullptr;
  ctx->d_coop_parts = nullptr;
  ctx->d_coop_phist = nullptr;
  ctx->d_coop_srec = nullptr;
  ctx->d_tables = nullptr;
  ctx->tables_words = 0;
  ctx->d_win = nullptr;
  ctx->win_bytes = 0;
  ctx->d_state_bak = nullptr;
  ctx->state_bak_bytes = 0;
  ctx->d_pct = nullptr;
  ctx->pct_words = 0;
  ctx->pct_valid = false;
  ctx->pc_node = -1;   // a deferred assume onto the freed state
  ctx->d_coop_notables = nullptr;
  ctx->coop_cfg_N = -1;
  ctx->coop_gen = 0;
  ctx->coop_dirty = true;
  ctx->d_ev = nullptr;
  ctx->ev_bytes = 0;
  ctx->ev_clean = false;
  ctx->d_ev_prof = nullptr;
  ctx->d_ev_pl = nullptr;
  ctx->ev_prof_dirty = true;
  ctx->d_srv = nullptr;   // (the server was stopped before anything freed)
  ctx->d_btab = nullptr;
  ctx->btab_cap = 0;
}

// ---- per-kernel timing -------------------------------------------------------
const char* kKernelNames[KSG_NKERNELS] = {"ksg_queue_kernel", "ksg_queue_topo_kernel", "ksg_batch_phase1",
                                          "ksg_batch_topk", "ksg_batch_phase2s", "ksg_sweep_static",
                                          "ksg_sweep", "ksg_topo_coop", "ksg_sweep_narrow",
                                          "ksg_capture_eval", "ksg_capture_norm", "ksg_eval_cycle",
                                          "ksg_batch_phase2v", "ksg_topo_coop_window"};

int tmark(ksg_ctx* ctx) {
  if (!ctx->timing) return KSG_OK;
  if (ctx->tev_used == (int)ctx->tev.size()) {
    hipEvent_t e;
    HIPC(ctx, hipEventCreate(&e));
    ctx->tev.push_back(e);
  }
  HIPC(ctx, hipEventRecord(ctx->tev[ctx->tev_used++], ctx->stream));
  return KSG_OK;
}

int tlaunched(ksg_ctx* ctx, int kind, double units) {
  if (!ctx->timing) return KSG_OK;
  ctx->tlaunch.emplace_back(kind, units);
  return tmark(ctx);
}

void treset(ksg_ctx* ctx) {
  ctx->tev_used = 0;
  ctx->tlaunch.clear();
  for (int k = 0; k < KSG_NKERNELS; k++) {
    ctx->kstat_ms[k] = 0;
    ctx->kstat_units[k] = 0;
    ctx->kstat_calls[k] = 0;
  }
}

// after the stream has been synchronised
int tcollect(ksg_ctx* ctx) {
  if (!ctx->timing) return KSG_OK;
  for (size_t i = 0; i < ctx->tlaunch.size() && (int)i + 1 < ctx->tev_used; i++) {
    float ms = 0;
    HIPC(ctx, hipEventElapsedTime(&ms, ctx->tev[i], ctx->tev[i + 1]));
    const int k = ctx->tlaunch[i].first;
    ctx->kstat_ms[k] += ms;
    ctx->kstat_units[k] += ctx->tlaunch[i].second;
    ctx->kstat_calls[k] += 1;
  }
  return KSG_OK;
}

bool profile_has(const ksg_profile& prof, int pl) {
  if ((prof.score_mask >> pl) & 1u) return true;
  for (int k = 0; k < prof.n_filter; k++)
    if (prof.filter_order[k] == pl) return true;
  return false;
}

// Does any pod of [first, first+count) need the PodTopologySpread /
// InterPodAffinity kernel under this profile?
bool needs_topo(ksg_ctx* ctx, const ksg_profile& prof, int first, int count) {
  const bool pts = profile_has(prof, KSG_PL_POD_TOPOLOGY_SPREAD), ipa = profile_has(prof, KSG_PL_INTER_POD_AFFINITY);
  if (!pts && !ipa) return false;
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if ((pts && p.pts >= 0) || (ipa && p.ipa >= 0)) return true;
  }
  return false;
}

int launch_queue(ksg_ctx* ctx, QueueArgs& a, int n_replicas, int block, bool topo) {
  (void)hipGetLastError();
  treset(ctx);
  HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  int rc;
  if ((rc = tmark(ctx))) return rc;
  if (topo) {
    if (block == 1024)
      hipLaunchKernelGGL(ksg_queue_topo_kernel<1024>, dim3(n_replicas), dim3(1024), 0, ctx->stream, a);
    else if (block == 512)
      hipLaunchKernelGGL(ksg_queue_topo_kernel<512>, dim3(n_replicas), dim3(512), 0, ctx->stream, a);
    else
      hipLaunchKernelGGL(ksg_queue_topo_kernel<256>, dim3(n_replicas), dim3(256), 0, ctx->stream, a);
  } else {
    if (block == 1024)
      hipLaunchKernelGGL(ksg_queue_kernel<1024>, dim3(n_replicas), dim3(1024), 0, ctx->stream, a);
    else if (block == 512)
      hipLaunchKernelGGL(ksg_queue_kernel<512>, dim3(n_replicas), dim3(512), 0, ctx->stream, a);
    else
      hipLaunchKernelGGL(ksg_queue_kernel<256>, dim3(n_replicas), dim3(256), 0, ctx->stream, a);
  }
  HIPC(ctx, hipGetLastError());
  if ((rc = tlaunched(ctx, topo ? KSG_K_QUEUE_TOPO : KSG_K_QUEUE, (double)n_replicas * a.count * a.c.N))) return rc;
  HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  return KSG_OK;
}

// Stop the persistent per-cycle server, if one runs: a stop call through the
// mailbox, then the stream drains.  Everything that puts work on the
// context's stream or reads / replaces node state calls this first (the
// server holds the node columns in registers while it runs).
// Whether [p, p + len) lies in a writable mapping of this process
// (/proc/self/maps): a device allocation the CPU may store to (large BAR)
// rather than a GPU-only virtual range.
// Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) unless the
// process set it: the batched walk dispatches one single-workgroup kernel per
// 64-pod batch, and reading each argument block from host memory at dispatch
// cost 8-16 % of the headline (scripts/gpu_kernarg_ab.sh, round 6).  The
// runtime reads its environment at the first HIP call, after this library is
// loaded in the Go shim and in native.py (which sets the same default).
__attribute__((constructor)) void ksg_env_defaults() { setenv("HIP_FORCE_DEV_KERNARG", "1", 0); }

bool host_writable(const void* p, size_t len) {
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + len;
  char line[512];
  bool ok = false;
  while (std::fgets(line, sizeof line, f)) {
    unsigned long lo = 0, hi = 0;
    char perm[8] = {0};
    if (std::sscanf(line, "%lx-%lx %7s", &lo, &hi, perm) != 3) continue;
    if (a >= lo && b <= hi) {
      ok = perm[0] == 'r' && perm[1] == 'w';
      break;
    }
  }
  std::fclose(f);
  return ok;
}

// At most one persistent per-cycle server per process.  Two contexts' servers
// alive together, one of them idling towards its exit while the other context
// starts its own, faulted a GPU test sequence (round 6, tests/test_gpu_eval.py
// with the module engine's server outliving its test; not reproduced with the
// servers serialised).  A context starting its server stops the other's first,
// under a process-wide lock that every server call holds from its post to its
// completion, so no call of the other context is in flight.
std::recursive_mutex g_srv_mu;
ksg_ctx* g_srv_ctx = nullptr;

int srv_stop(ksg_ctx* ctx) {
  std::lock_guard<std::recursive_mutex> lk(g_srv_mu);
  if (ctx && g_srv_ctx == ctx) g_srv_ctx = nullptr;
  if (!ctx || !ctx->srv_running) return KSG_OK;
  ctx->srv_running = false;
  SrvMailbox* mb = ctx->h_mb;
  mb->k.op = 1;
  const unsigned seq = ++ctx->ev_seq == 0 ? ++ctx->ev_seq : ctx->ev_seq;
  __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

int check_ready(ksg_ctx* ctx) {
  if (!ctx) return KSG_E_INVALID;
  if (!ctx->have_nodes || !ctx->have_wl || !ctx->have_prof)
    return fail(ctx, KSG_E_STATE, "profile, nodes and workload must be loaded first");
  return KSG_OK;
}

// Pods [first, first + count) are staged into LDS by the evaluating kernels:
// each one's program blob must fit.  Checked per evaluated range, so one
// oversized pod refuses only its own evaluations (commits read programs from
// global memory and need no LDS).
int check_blobs(ksg_ctx* ctx, int first, int count) {
  for (int i = first; i < first + count; i++)
    if (ctx->h_pods[i].blob_len > KSG_BLOB_MAX)
      return fail(ctx, KSG_E_UNSUPPORTED, "pod " + std::to_string(i) + ": program blob exceeds the LDS budget");
  return KSG_OK;
}

// Host mirror of layout_slots(): words of LDS histograms a pod needs.
int topo_words(ksg_ctx* ctx, const ksg_pod& p, bool pts, bool ipa) {
  const std::vector<int32_t>& P = ctx->h_prog;
  int words = 0;
  auto slot = [&](int col, bool mark) {
    if (col < 0 || col >= std::max(ctx->c.L, 1)) { words = 1 << 30; return; }
    if (ctx->h_col_unique[col]) return;
    const int V = ctx->h_col_vocab[col];
    words += V + (V + 31) / 32 * (mark ? 2 : 1);
  };
  if (pts && p.pts >= 0) {
    const int nh = P[p.pts], ns = P[p.pts + 1];
    if (nh > ksg::kMaxHard || ns > ksg::kMaxSoft) return 1 << 30;
    for (int i = 0; i < nh; i++) slot(P[p.pts + 3 + 7 * i], false);
    for (int i = 0; i < ns; i++) slot(P[p.pts + 3 + 7 * nh + 6 * i], true);
  }
  if (ipa && p.ipa >= 0) {
    size_t w = p.ipa;
    const int na = P[w];
    if (na > ksg::kMaxAff) return 1 << 30;
    for (int i = 0; i < na; i++) slot(P[w + 3 + i], false);
    w += 3 + na;
    const int nn = P[w++];
    if (nn > ksg::kMaxAnti) return 1 << 30;
    for (int i = 0; i < nn; i++) slot(P[w + 2 * i], false);
    w += 2 * nn;
    const int np = P[w++];
    if (np > ksg::kMaxPref) return 1 << 30;
    for (int i = 0; i < np; i++) slot(P[w + 3 * i], false);
  }
  return words;
}

// Refuse inputs outside what the kernels implement instead of computing
// something else.
int check_supported(ksg_ctx* ctx, const ksg_profile& prof, int first, int count) {
  const bool pts = profile_has(prof, KSG_PL_POD_TOPOLOGY_SPREAD), ipa = profile_has(prof, KSG_PL_INTER_POD_AFFINITY);
  if (!pts && !ipa) return KSG_OK;
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if (topo_words(ctx, p, pts, ipa) > KSG_HIST_MAX)
      return fail(ctx, KSG_E_UNSUPPORTED,
                  "pod " + std::to_string(i) + ": topology terms exceed the LDS histogram budget");
  }
  return KSG_OK;
}

// The batched path covers node-local plugins only and packs raw scores into
// 8-byte records; use it only when the values provably fit.
// Any pod of [first, first + count) with host ports (NodePorts reads and its
// assume writes the node's UsedPorts: the queue kernels and the per-cycle
// path model that; the batched, sweep and chip-wide topology paths do not).
// Pods with claims (a volume program) take the same paths: only the queue
// kernels' evaluator (eval_node_src) runs the volume plugins' Filter.
bool range_has_ports(const ksg_ctx* ctx, int first, int count) {
  for (int i = first; i < first + count; i++)
    if (ctx->h_pods[i].ports >= 0 || ctx->h_pods[i].vol >= 0) return true;
  return false;
}

bool batch_eligible(ksg_ctx* ctx, int first, int count) {
  const ksg_profile& prof = ctx->prof;
  if (needs_topo(ctx, prof, first, count)) return false;
  if (range_has_ports(ctx, first, count)) return false;
  if (ctx->c.T > 255) return false;
  if (ctx->c.N > (1 << 19)) return false;   // changed-node bitmap must fit LDS
  int64_t wsum = 0;
  for (int pl : {KSG_PL_NODE_RESOURCES_FIT, KSG_PL_BALANCED_ALLOCATION, KSG_PL_IMAGE_LOCALITY})
    if ((prof.score_mask >> pl) & 1u) {
      if (prof.weight[pl] < 0) return false;
      wsum += prof.weight[pl];
    }
  if (wsum * 100 >= (1ll << 31)) return false;
  for (int i = first; i < first + count; i++)
    if (ctx->h_na_pref_sum[i] > 0xffff || ctx->h_na_pref_sum[i] < 0) return false;
  return true;
}

QueueArgs base_args(ksg_ctx* ctx) {
  QueueArgs a{};
  a.c = ctx->c;
  a.st = ctx->st;
  a.pods = ctx->d_pods;
  a.prog = ctx->d_prog;
  return a;
}

struct Tmp {
  std::vector<void*> ptrs;
  ~Tmp() { for (void* p : ptrs) (void)hipFree(p); }
  template <typename T>
  hipError_t alloc(T** p, size_t bytes) {
    hipError_t e = hipMalloc((void**)p, std::max<size_t>(bytes, 8));
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
};
#define TA(tmp, p, bytes)                                                              \
  do {                                                                                 \
    hipError_t _e = (tmp).alloc((p), (bytes));                                         \
    if (_e != hipSuccess) return fail(ctx, KSG_E_NOMEM, hipGetErrorString(_e));        \
  } while (0)

// ksg_batch_phase2s instances: (RM 4 | KSG_MAX_RES | 4 with N32) x (64 | 128 lanes)
static const std::array<const void*, 6>& slot_kernels() {
  static const std::array<const void*, 6> k = {
      (const void*)ksg_batch_phase2s<4, 64>,           (const void*)ksg_batch_phase2s<4, 128>,
      (const void*)ksg_batch_phase2s<KSG_MAX_RES, 64>, (const void*)ksg_batch_phase2s<KSG_MAX_RES, 128>,
      (const void*)ksg_batch_phase2s<4, 64, true>,     (const void*)ksg_batch_phase2s<4, 128, true>};
  return k;
}
// index into slot_kernels(): the instance for (n32, RM, lanes <= 128)
static int slot_kernel_index(bool n32, int slot_rm, int lanes) {
  return (n32 ? 4 : slot_rm == 4 ? 0 : 2) + (lanes <= 64 ? 0 : 1);
}

bool profile_cm_fast(const ksg_profile& prof);

// Host half of the N32 check for a batched run of pods [first, first + count)
// (the node half is ksg_range32): the profile scores Fit / BalancedAllocation
// over exactly {cpu, memory} and filters with Fit for every pod (so the Fit
// filter bounds every requested sum by the allocatable), the pods' memory
// quantities are whole MiB and their cpu fits 30 bits, Fit's weights keep
// the weighted numerator below 2^30.  Fills the pods' non-zero excess bounds.
bool range32_candidate(ksg_ctx* ctx, int first, int count, int64_t* xc, int64_t* xm, bool mw = false) {
  const ksg_profile& prof = ctx->prof;
  if (!profile_cm_fast(prof) || ctx->c.R > 4 || ctx->force_path == 3) return false;
  bool fit = false;
  for (int k = 0; k < prof.n_filter; k++) fit |= prof.filter_order[k] == KSG_PL_NODE_RESOURCES_FIT;
  if (!fit || (prof.fit_w[0] + prof.fit_w[1]) * 100 >= (1 << 30)) return false;
  int64_t wsum = 0;   // the slot walk's weighted totals in 32 bits
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    if ((prof.score_mask >> pl) & 1u) {
      if (prof.weight[pl] < 0) return false;
      wsum += prof.weight[pl];
    }
  if (wsum * 100 >= (1 << 30)) return false;
  constexpr int64_t kMiB = 1 << 20, k46 = (int64_t)1 << 46;
  *xc = *xm = 0;
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if ((p.filter_skip >> KSG_PL_NODE_RESOURCES_FIT) & 1u) return false;
    const int64_t rc = p.req[KSG_RES_CPU], rm = p.req[KSG_RES_MEM];
    if (rc < 0 || rm < 0 || p.nz_cpu < 0 || p.nz_mem < 0) return false;
    if (rc >= (1 << 30) || p.nz_cpu >= (1 << 30)) return false;
    if (mw) {   // the wide-memory instance: bytes, below 2^46
      if (rm >= k46 || p.nz_mem >= k46) return false;
      *xm = std::max(*xm, p.nz_mem - rm);
    } else {
      if (((rm | p.nz_mem) & (kMiB - 1)) || (rm >> 20) >= (1 << 30) || (p.nz_mem >> 20) >= (1 << 30)) return false;
      *xm = std::max(*xm, (p.nz_mem - rm) >> 20);
    }
    *xc = std::max(*xc, p.nz_cpu - rc);
  }
  return true;
}

// 32-bit Fit / BalancedAllocation in the slot walk when the ranges allow (one
// small check launch + a 4-byte read per call).
int decide_n32(ksg_ctx* ctx, int32_t first, int32_t count, bool* n32) {
  *n32 = false;
  int64_t xc = 0, xm = 0;
  if (ctx->c.R <= 4 && range32_candidate(ctx, first, count, &xc, &xm)) {
    if (!ctx->d_flag) {
      int rc;
      if ((rc = dalloc(ctx, &ctx->d_flag, 4))) return rc;
    }
    HIPC(ctx, hipMemsetAsync(ctx->d_flag, 0, 16, ctx->stream));
    hipLaunchKernelGGL(ksg_range32, dim3((ctx->c.N + 255) / 256), dim3(256), 0, ctx->stream, ctx->c, ctx->st, xc, xm,
                       count, 0, ctx->d_flag);
    unsigned bad = 0;
    HIPC(ctx, hipMemcpyAsync(&bad, ctx->d_flag, sizeof(bad), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(ctx, hipStreamSynchronize(ctx->stream));
    *n32 = bad == 0;
  }
  ctx->last_n32 = *n32;
  return KSG_OK;
}

// The wide-memory scope of the speculate-and-verify walk: the N32 check's cpu
// half, memory in bytes (ksg_range32 mw = 1).
int decide_mw(ksg_ctx* ctx, int32_t first, int32_t count, bool* mw) {
  *mw = false;
  int64_t xc = 0, xm = 0;
  if (ctx->c.R <= 4 && ctx->force_path != 3 && range32_candidate(ctx, first, count, &xc, &xm, true)) {
    if (!ctx->d_flag) {
      int rc;
      if ((rc = dalloc(ctx, &ctx->d_flag, 4))) return rc;
    }
    HIPC(ctx, hipMemsetAsync(ctx->d_flag, 0, 16, ctx->stream));
    hipLaunchKernelGGL(ksg_range32, dim3((ctx->c.N + 255) / 256), dim3(256), 0, ctx->stream, ctx->c, ctx->st, xc, xm,
                       count, 1, ctx->d_flag);
    unsigned bad = 0;
    HIPC(ctx, hipMemcpyAsync(&bad, ctx->d_flag, sizeof(bad), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(ctx, hipStreamSynchronize(ctx->stream));
    *mw = bad == 0;
  }
  return KSG_OK;
}

// LDS budget attribute of the phase-2 instances (once per process)
int set_phase2_attrs(ksg_ctx* ctx, size_t budget) {
  int rc;
  for (const void* f : slot_kernels())
    if ((rc = func_lds_attr(ctx, f, budget))) return rc;
  return KSG_OK;
}

constexpr size_t kSpecLds = 130 * 1024;   // ... of the speculate-and-verify walk (static part ~16 KB): the
                                          // launch always asks for all of it, so that no other kernel's
                                          // workgroup shares the walk's CU

// Host half of the speculate-and-verify walk's scope (ksched_phase2v.h): on top
// of the N32 check, every weighted total fits the column word's 27 bits.
bool spec_candidate(const ksg_ctx* ctx) {
  int64_t wsum = 0;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    if ((ctx->prof.score_mask >> pl) & 1u) wsum += ctx->prof.weight[pl];
  return ctx->c.R <= 4 && wsum * 100 < (1 << kSvTotalBits);
}

int run_batched(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* d_pl, ksg_result* d_res, const CapArgs* cap,
                const ksg_profile* d_prof) {
  const int N = ctx->c.N;
  // the slot walk, one launch chain per batch (captured queues, the "slot"
  // mode, the window pipeline off)
  if (!ctx->d_rec) {
    int rc;
    if ((rc = dalloc(ctx, &ctx->d_rec, (size_t)KSG_BATCH_MAX * N))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_img, (size_t)KSG_BATCH_MAX * N))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_stat, (size_t)KSG_BATCH_MAX * N))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_pmax, (size_t)2 * KSG_BATCH_MAX))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_p1, (size_t)KSG_BATCH_MAX))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_top, (size_t)KSG_BATCH_MAX * KSG_BATCH_MAX))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_pmax, 0, sizeof(int32_t) * 2 * KSG_BATCH_MAX, ctx->stream));
  }
  BatchArgs b{};
  b.c = ctx->c;
  b.st = ctx->st;
  b.pods = ctx->d_pods;
  b.prog = ctx->d_prog;
  b.prof = d_prof;
  b.rec = ctx->d_rec;
  b.img = ctx->d_img;
  b.pmax = ctx->d_pmax;
  b.p1 = ctx->d_p1;
  b.top = ctx->d_top;
  b.placements = d_pl;
  b.results = d_res;
#ifdef KSG_STAMPS
  if (!ctx->d_stamps) {
    int rc;
    if ((rc = dalloc(ctx, &ctx->d_stamps, 16))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_stamps, 0, 128, ctx->stream));
  }
  b.stamps = ctx->d_stamps;
#endif
  // Plan batches so that phase 2's LDS preload (changed-node bitmap + pod
  // records + the program range of the batch + one slot of live resource
  // columns per pod) fits the dynamic LDS budget.
  constexpr size_t kLdsBudget = 120 * 1024;
  const size_t cm_words = (size_t)((((N + 31) / 32) + 3) & ~3);
  const int slot_rm = ctx->c.R <= 4 ? 4 : KSG_MAX_RES;   // ksg_batch_phase2s<RM> instance
  const size_t slot_bytes = 8 * (size_t)(2 * slot_rm + 10);   // SlotLayout<RM>::STRIDE int64 words
  {
    int rc;
    if ((rc = set_phase2_attrs(ctx, kLdsBudget))) return rc;
  }
  bool n32 = false;
  {
    int rc;
    if ((rc = decide_n32(ctx, first, count, &n32))) return rc;
  }
  b.stat = n32 ? ctx->d_stat : nullptr;
  ctx->last_spec = false;
  ctx->last_mw = false;
  (void)hipGetLastError();
  treset(ctx);
  HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  int trc;
  if ((trc = tmark(ctx))) return trc;
  for (int off = 0; off < count;) {
    int nb = std::min(ctx->slot_block, count - off);
    int64_t lo = 0, hi = 0;
    size_t bytes = 0;
    const size_t budget = kLdsBudget;
    for (;;) {
      lo = ctx->h_pods[first + off].blob;
      hi = lo;
      for (int k = 0; k < nb; k++) {
        const ksg_pod& q = ctx->h_pods[first + off + k];
        lo = std::min<int64_t>(lo, q.blob);
        hi = std::max<int64_t>(hi, (int64_t)q.blob + q.blob_len);
      }
      const size_t words = (cm_words + (size_t)nb * (sizeof(ksg_pod) / 4) + (size_t)(hi - lo) + 3) & ~(size_t)3;
      bytes = 4 * words + (size_t)nb * slot_bytes;   // + one live slot row per pod
      if (bytes <= budget || nb == 1) break;
      nb = std::max(1, nb / 2);
    }
    if (bytes > budget) return fail(ctx, KSG_E_UNSUPPORTED, "batch does not fit the LDS budget");
    b.b0 = first + off;
    b.out0 = off;
    b.nb = nb;
    b.prog_lo = (int32_t)lo;
    b.prog_len = (int32_t)(hi - lo);
    const double units = (double)b.nb * N;   // (pod, node) pairs of the batch
    hipLaunchKernelGGL(ksg_batch_phase1, dim3((N + 255) / 256, b.nb), dim3(256), 0, ctx->stream, b);
    if ((trc = tlaunched(ctx, KSG_K_BATCH_PHASE1, units))) return trc;
    hipLaunchKernelGGL(ksg_batch_topk<1024>, dim3(b.nb), dim3(1024), 0, ctx->stream, b);
    if ((trc = tlaunched(ctx, KSG_K_BATCH_TOPK, units))) return trc;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(BatchArgs)>(
                           const_cast<void*>(slot_kernels()[slot_kernel_index(n32, slot_rm, ctx->slot_block)])),
                       dim3(1), dim3(ctx->slot_block), bytes, ctx->stream, b);
    if ((trc = tlaunched(ctx, KSG_K_BATCH_PHASE2S, 0.5 * b.nb * (b.nb + 1)))) return trc;
    if (cap) {   // the batch's capture, on the post-batch state (ksched_capture.h)
      CapArgs ca = *cap;
      ca.b0 = b.b0;
      ca.nb = b.nb;
      ca.out0 = b.out0;
      ca.rec = ctx->d_rec;
      HIPC(ctx, hipMemsetAsync(ca.stats, 0, sizeof(int32_t) * 4 * b.nb, ctx->stream));
      hipLaunchKernelGGL(ksg_capture_eval, dim3((N + 255) / 256, b.nb), dim3(256), 0, ctx->stream, ca);
      if ((trc = tlaunched(ctx, KSG_K_CAPTURE_EVAL, units))) return trc;
      hipLaunchKernelGGL(ksg_capture_norm, dim3((N + 255) / 256, b.nb), dim3(256), 0, ctx->stream, ca);
      if ((trc = tlaunched(ctx, KSG_K_CAPTURE_NORM, units))) return trc;
    }
    off += nb;
  }
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  return KSG_OK;
}

// The window pipeline with the persistent spec walk (ksg_batch_phase2v_run):
// the batch table first (the same LDS-fitting batches as the per-batch
// launches), the walk launched once on the main stream, then phase 1 / top-k
// of batch b on the second stream as soon as the walk has finished batch
// b - 2 (the walk's counter in pinned host memory; each of those launches
// acquires at its dispatch what the walk released).  The walk polls each
// batch's top-k flag as before.  The host's wait is bounded: a walk that
// ended early (a timed-out hand-off, a broken invariant) stops the launches
// and run_internal reports its words.
int state_copy(ksg_ctx* ctx, bool save);

int run_spec_persistent(ksg_ctx* ctx, const BatchArgs& b0, int32_t first, int32_t count, size_t cm_words, bool mw,
                        unsigned* tk, int32_t* carry_n) {
  const int N = ctx->c.N;
  constexpr int B = 64;
  std::vector<int32_t>& tab = ctx->h_btab;
  tab.clear();
  for (int off = 0, prev_nb = 0; off < count;) {
    int nb = std::min(B, count - off);
    int64_t lo = 0, hi = 0;
    size_t bytes = 0;
    for (;;) {
      lo = ctx->h_pods[first + off].blob;
      hi = lo;
      for (int k = 0; k < nb; k++) {
        const ksg_pod& q = ctx->h_pods[first + off + k];
        lo = std::min<int64_t>(lo, q.blob);
        hi = std::max<int64_t>(hi, (int64_t)q.blob + q.blob_len);
      }
      bytes = 4 * ((cm_words + (size_t)nb * (sizeof(ksg_pod) / 4) + (size_t)(hi - lo) + 3) & ~(size_t)3) +
              (size_t)kSvSlots * kSvRow * 8 + (size_t)kSvSlots * 64 * 4 + (size_t)64 * (nb + prev_nb) * 4;
      if (bytes <= kSpecLds || nb == 1) break;
      nb = std::max(1, nb / 2);
    }
    if (bytes > kSpecLds) return fail(ctx, KSG_E_UNSUPPORTED, "batch does not fit the LDS budget");
    for (int32_t v : {first + off, off, nb, (int32_t)lo, (int32_t)(hi - lo), prev_nb}) tab.push_back(v);
    prev_nb = nb;
    off += nb;
  }
  const int nbatch = (int)(tab.size() / 6);
  int rc;
  if (tab.size() > ctx->btab_cap) {
    if (ctx->d_btab) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)ctx->d_btab);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipFree(ctx->d_btab);
      ctx->d_btab = nullptr;
    }
    if ((rc = dalloc(ctx, &ctx->d_btab, tab.size()))) return rc;
    ctx->btab_cap = tab.size();
  }
  if (!ctx->h_p2done) {
    HIPC(ctx, hipHostMalloc((void**)&ctx->h_p2done, 64, hipHostMallocMapped | hipHostMallocCoherent));
    void* dp = nullptr;
    HIPC(ctx, hipHostGetDevicePointer(&dp, ctx->h_p2done, 0));
    ctx->d_p2done = static_cast<unsigned*>(dp);
  }
  hipStream_t s1 = ctx->stream2, s2 = ctx->stream;
  // the pre-call state, for a walk whose top-k poll gives up (run_internal
  // restores it and runs the per-batch form)
  if ((rc = state_copy(ctx, true))) return rc;
  ctx->last_persist = true;
  HIPC(ctx, hipMemcpyAsync(ctx->d_btab, tab.data(), sizeof(int32_t) * tab.size(), hipMemcpyHostToDevice, s2));
  if (ctx->inject_timeout & 16) {   // test injection: the walk finds its poll's give-up word set after batch 0
    ctx->inject_timeout &= ~16;
    HIPC(ctx, hipMemsetAsync(tk + 2, 0x01, 1, s2));
  }
  volatile unsigned* done = ctx->h_p2done;
  *done = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  SpecRun r{};
  r.btab = ctx->d_btab;
  r.nbatch = nbatch;
  for (int q = 0; q < 2; q++) {
    r.rec[q] = ctx->d_prec[q];
    r.img[q] = ctx->d_pimg[q];
    r.rect[q] = ctx->d_prect[q];
    r.imgt[q] = ctx->d_pimgt[q];
    r.pmax[q] = ctx->d_ppmax[q];
    r.p1[q] = ctx->d_pp1[q];
    r.top[q] = ctx->d_ptop[q];
  }
  r.carry = ctx->d_carry;
  r.carry_n = carry_n;
  r.done = ctx->d_p2done;
  BatchArgs base = b0;
  base.tk_arrive = tk;
  base.tk_done = tk + 1;
  base.tk_timeout = tk + 2;
  base.walk_err = tk + 3;
  base.inject_walk_err = ctx->inject_walk_err;
  base.tk_sc = 1;
  base.stat = nullptr;
  base.xcd_grid = 1;
  const void* run_kern = mw ? (const void*)ksg_batch_phase2v_run<64 * kSvWaves, true>
                            : (const void*)ksg_batch_phase2v_run<64 * kSvWaves, false>;
  if ((rc = func_lds_attr(ctx, run_kern, kSpecLds))) return rc;
  void* kargs[] = {&base, &r};
  HIPC(ctx, hipLaunchKernel(run_kern, dim3(1), dim3(64 * kSvWaves), kargs, kSpecLds, s2));
  const auto t0 = std::chrono::steady_clock::now();
  for (int bi = 0; bi < nbatch; bi++) {
    if (bi >= 2) {   // phase 1 of batch bi reads what the walk of batch bi - 2 wrote, into its buffers
      for (unsigned spins = 0; *done < (unsigned)(bi - 1); spins++) {
        __builtin_ia32_pause();
        if ((spins & 4095) == 4095) {
          const hipError_t e = hipStreamQuery(s2);
          if (e != hipErrorNotReady && *done < (unsigned)(bi - 1)) {
            if (e != hipSuccess) return fail(ctx, KSG_E_DEVICE, std::string("spec walk: ") + hipGetErrorString(e));
            bi = nbatch;   // the walk ended early: run_internal reports its words
            break;
          }
          if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 120.0)
            return fail(ctx, KSG_E_DEVICE, "spec walk: no progress for 120 s");
        }
      }
      if (bi >= nbatch) break;
    }
    const int32_t* d = tab.data() + 6 * bi;
    const int par = bi & 1;
    BatchArgs b = base;
    b.b0 = d[0];
    b.out0 = d[1];
    b.nb = d[2];
    b.prog_lo = d[3];
    b.prog_len = d[4];
    b.k_extra = d[5];
    b.rec = r.rec[par];
    b.img = r.img[par];
    b.rect = r.rect[par];
    b.imgt = r.imgt[par];
    b.pmax = r.pmax[par];
    b.p1 = r.p1[par];
    b.top = r.top[par];
    b.carry = r.carry + (par ^ 1) * KSG_BATCH_MAX;
    b.carry_n = carry_n + (par ^ 1);
    b.carry_out = r.carry + par * KSG_BATCH_MAX;
    b.carry_out_n = carry_n + par;
    b.tk_seq = (unsigned)bi + 1;
    hipLaunchKernelGGL(ksg_batch_phase1, dim3(((((N + 255) / 256) + 7) & ~7) * b.nb), dim3(256), 0, s1, b);
    hipLaunchKernelGGL(ksg_batch_topk<1024>, dim3(b.nb), dim3(1024), 0, s1, b);
  }
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipEventRecord(ctx->ev1, s2));
  return KSG_OK;
}

// Pipelined batched path (the two-batch window).  Batch b's phase 1 + top-k run on
// a second stream while batch b - 1's phase 2 runs: phase 1 of batch b reads
// the state at least as of the end of batch b - 2 (it waits for that phase 2),
// and phase 2 of batch b carries batch b - 1's changed nodes as changed slots
// (the two-batch window; top sets hold k_extra = |batch b - 1| extra keys).
// With per-kernel timing on, every launch goes to one stream (same
// arithmetic, no overlap) so that each launch is timed on its own.
int run_pipe(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* d_pl, ksg_result* d_res, const ksg_profile* d_prof) {
  const int N = ctx->c.N;
  int rc;
  ctx->last_spec = false;
  ctx->last_mw = false;
  ctx->last_persist = false;
  if (!ctx->d_prec[0]) {
    for (int q = 0; q < 2; q++) {
      if ((rc = dalloc(ctx, &ctx->d_prec[q], (size_t)KSG_BATCH_MAX * N))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_pimg[q], (size_t)KSG_BATCH_MAX * N))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_pstat[q], (size_t)KSG_BATCH_MAX * N))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_ppmax[q], (size_t)2 * KSG_BATCH_MAX))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_pp1[q], (size_t)KSG_BATCH_MAX))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_ptop[q], (size_t)KSG_BATCH_MAX * KSG_BATCH_MAX))) return rc;
      HIPC(ctx, hipMemsetAsync(ctx->d_ppmax[q], 0, sizeof(int32_t) * 2 * KSG_BATCH_MAX, ctx->stream));
    }
    if ((rc = dalloc(ctx, &ctx->d_carry, (size_t)2 * KSG_BATCH_MAX + 6))) return rc;   // + carry_n[2], tk[4]
  }
  if (!ctx->stream2) {
    // the second stream at another priority than the main one: the runtime
    // keeps a queue pool per priority, so the two never share a hardware
    // queue, where the persistent walk would sit in front of the phase 1 /
    // top-k launches it waits for
    int least = 0, greatest = 0;
    HIPC(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPC(ctx, hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, greatest));
    for (int q = 0; q < 2; q++) {
      HIPC(ctx, hipEventCreateWithFlags(&ctx->ev_tk[q], hipEventDisableTiming));
      HIPC(ctx, hipEventCreateWithFlags(&ctx->ev_p2[q], hipEventDisableTiming));
    }
  }
  int32_t* carry_n = ctx->d_carry + 2 * KSG_BATCH_MAX;   // [2]
  unsigned* tk = reinterpret_cast<unsigned*>(carry_n + 2);   // top-k hand-off: arrive, done, timeout
  ctx->pipe_tk = tk;
  HIPC(ctx, hipMemsetAsync(carry_n, 0, 6 * sizeof(int32_t), ctx->stream));   // carry_n, tk[0..3]
  const bool window = ctx->pipe_window != 0;
  const bool overlap = window && !ctx->timing && ctx->pipe_overlap;
  const int slot_rm = ctx->c.R <= 4 ? 4 : KSG_MAX_RES;
  // mode 4: the slot walk inside this pipeline (one lane per slot).  (The
  // round-2 two-version walk, a round-3 one-wave walk with two slots per lane
  // and the transposed walk, all measured no faster, were removed.)
  bool n32 = false, mw = false;
  if (ctx->batch_mode >= 4 && (rc = decide_n32(ctx, first, count, &n32))) return rc;
  // mode 6: the speculate-and-verify walk (ksched_phase2v.h), N32 scope, 64-pod
  // batches; memory outside the N32 ranges (not whole MiB, as kubelets report
  // it, or too large) takes its wide-memory instance (MW: memory in int64
  // bytes, the same quotients)
  if (ctx->batch_mode == 6 && window && !n32 && spec_candidate(ctx) && (rc = decide_mw(ctx, first, count, &mw)))
    return rc;
  const bool specw = ctx->batch_mode == 6 && window && (n32 || mw) && spec_candidate(ctx);
  ctx->last_spec = specw;
  ctx->last_mw = specw && mw;
  const void* spec_kern = mw ? (const void*)ksg_batch_phase2v<64 * kSvWaves, true>
                             : (const void*)ksg_batch_phase2v<64 * kSvWaves, false>;
  if (specw && !ctx->d_prect[0]) {   // the node-major copies phase 1 writes (records, ImageLocality)
    for (int q = 0; q < 2; q++) {
      if ((rc = dalloc(ctx, &ctx->d_prect[q], (size_t)64 * N))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_pimgt[q], (size_t)64 * N))) return rc;
    }
  }
  if (specw && (rc = func_lds_attr(ctx, spec_kern, kSpecLds))) return rc;
  // batches: 64 pods in the window (the spec walk, or the slot walk with the
  // previous batch's 64 slots carried beside this batch's), else slot_block
  const int B = specw || window ? 64 : ctx->slot_block;
  const int slots = window ? 2 * B : B;   // carried + this batch's slots
  const int sblock = slots <= 64 ? 64 : 128;
  const void* kern = slot_kernels()[slot_kernel_index(n32, slot_rm, sblock)];
  const int block = sblock;
  const size_t kLdsBudget = specw ? kSpecLds : 120 * 1024;
  const size_t slot_bytes = 8 * (size_t)(2 * slot_rm + 10);   // SlotLayout<RM>::STRIDE int64 words
  if ((rc = set_phase2_attrs(ctx, 120 * 1024))) return rc;   // the slot-walk instances (fallback)
  BatchArgs b{};
  b.c = ctx->c;
  b.st = ctx->st;
  b.pods = ctx->d_pods;
  b.prog = ctx->d_prog;
  b.prof = d_prof;
  b.placements = d_pl;
  b.results = d_res;
  const size_t cm_words = (size_t)((((N + 31) / 32) + 3) & ~3);
#ifdef KSG_STAMPS
  if (!ctx->d_stamps) {
    if ((rc = dalloc(ctx, &ctx->d_stamps, 16))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_stamps, 0, 128, ctx->stream));
  }
  b.stamps = ctx->d_stamps;
#endif
  hipStream_t s1 = overlap ? ctx->stream2 : ctx->stream, s2 = ctx->stream;
  (void)hipGetLastError();
  treset(ctx);
  HIPC(ctx, hipEventRecord(ctx->ev0, s2));
  if (overlap) HIPC(ctx, hipStreamWaitEvent(s1, ctx->ev0, 0));
  if ((rc = tmark(ctx))) return rc;
  if (specw && overlap && ctx->spec_persist)
    return run_spec_persistent(ctx, b, first, count, cm_words, mw, tk, carry_n);
  int prev_nb = 0;
  for (int off = 0, bi = 0; off < count; bi++) {
    const int par = bi & 1;
    int nb = std::min(B, count - off);
    int64_t lo = 0, hi = 0;
    size_t bytes = 0;
    for (;;) {
      lo = ctx->h_pods[first + off].blob;
      hi = lo;
      for (int k = 0; k < nb; k++) {
        const ksg_pod& q = ctx->h_pods[first + off + k];
        lo = std::min<int64_t>(lo, q.blob);
        hi = std::max<int64_t>(hi, (int64_t)q.blob + q.blob_len);
      }
      if (specw)   // row versions + T as node indices ([pod][nb + carried])
        bytes = 4 * ((cm_words + (size_t)nb * (sizeof(ksg_pod) / 4) + (size_t)(hi - lo) + 3) & ~(size_t)3) +
                (size_t)kSvSlots * kSvRow * 8 + (size_t)kSvSlots * 64 * 4 + (size_t)64 * (nb + prev_nb) * 4;
      else
        bytes = 4 * ((cm_words + (size_t)nb * (sizeof(ksg_pod) / 4) + (size_t)(hi - lo) + 3) & ~(size_t)3) +
                (size_t)sblock * slot_bytes;
      if (bytes <= kLdsBudget || nb == 1) break;
      nb = std::max(1, nb / 2);
    }
    if (bytes > kLdsBudget) return fail(ctx, KSG_E_UNSUPPORTED, "batch does not fit the LDS budget");
    b.b0 = first + off;
    b.out0 = off;
    b.nb = nb;
    b.prog_lo = (int32_t)lo;
    b.prog_len = (int32_t)(hi - lo);
    b.rec = ctx->d_prec[par];
    b.img = ctx->d_pimg[par];
    b.stat = n32 && !specw ? ctx->d_pstat[par] : nullptr;   // (the spec walk computes its statics)
    b.rect = specw ? ctx->d_prect[par] : nullptr;
    b.imgt = specw ? ctx->d_pimgt[par] : nullptr;
    b.xcd_grid = specw ? 1 : 0;
    b.pmax = ctx->d_ppmax[par];
    b.p1 = ctx->d_pp1[par];
    b.top = ctx->d_ptop[par];
    b.k_extra = window ? prev_nb : 0;
    b.carry = window ? ctx->d_carry + (par ^ 1) * KSG_BATCH_MAX : nullptr;
    b.carry_n = window ? carry_n + (par ^ 1) : nullptr;
    b.carry_out = window ? ctx->d_carry + par * KSG_BATCH_MAX : nullptr;
    b.carry_out_n = window ? carry_n + par : nullptr;
    const double units = (double)nb * N;
    // the walk waits for this batch's top-k: it polls a flag the last top-k
    // workgroup stores (no cross-stream event in front of it on the critical
    // stream)
    const bool tk_flag = overlap;
    b.tk_arrive = tk_flag ? tk : nullptr;
    b.tk_done = tk_flag ? tk + 1 : nullptr;
    b.tk_timeout = tk_flag ? tk + 2 : nullptr;
    b.walk_err = tk + 3;
    b.inject_walk_err = ctx->inject_walk_err;
    b.tk_seq = (unsigned)bi + 1;
    BatchArgs bt = b;   // the top-k launch: signals
    bt.tk_sc = specw && tk_flag ? 1 : 0;
    b.tk_sc = bt.tk_sc;
    // phase 1 of batch b reads the state as of the end of batch b - 2 at least,
    // and reuses the buffers phase 2 of batch b - 2 read
    if (overlap && bi >= 2) HIPC(ctx, hipStreamWaitEvent(s1, ctx->ev_p2[par], 0));
    if (specw)
      hipLaunchKernelGGL(ksg_batch_phase1, dim3(((((N + 255) / 256) + 7) & ~7) * nb), dim3(256), 0, s1, b);
    else
      hipLaunchKernelGGL(ksg_batch_phase1, dim3((N + 255) / 256, nb), dim3(256), 0, s1, b);
    if ((rc = tlaunched(ctx, KSG_K_BATCH_PHASE1, units))) return rc;
    hipLaunchKernelGGL(ksg_batch_topk<1024>, dim3(nb), dim3(1024), 0, s1, bt);
    if ((rc = tlaunched(ctx, KSG_K_BATCH_TOPK, units))) return rc;
    if (specw) {
      hipLaunchKernelGGL(reinterpret_cast<void (*)(BatchArgs)>(const_cast<void*>(spec_kern)), dim3(1),
                         dim3(64 * kSvWaves), kSpecLds, s2, b);
      if ((rc = tlaunched(ctx, KSG_K_BATCH_PHASE2V, 0.5 * nb * (nb + 1)))) return rc;
    } else {
      hipLaunchKernelGGL(reinterpret_cast<void (*)(BatchArgs)>(const_cast<void*>(kern)), dim3(1), dim3(block), bytes, s2, b);
      if ((rc = tlaunched(ctx, KSG_K_BATCH_PHASE2S, 0.5 * nb * (nb + 1)))) return rc;
    }
    if (overlap) HIPC(ctx, hipEventRecord(ctx->ev_p2[par], s2));
    prev_nb = nb;
    off += nb;
  }
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipEventRecord(ctx->ev1, s2));
  return KSG_OK;
}

// The replica sweep packs the replica-independent plugin results into 8-byte
// static records and the per-replica result into pack_rec(); use it when
// every replica profile is node-local and the values provably fit.
bool sweep_eligible(ksg_ctx* ctx, const ksg_profile* profiles, int R, int first, int count) {
  if (ctx->c.T > 255) return false;
  if (range_has_ports(ctx, first, count)) return false;
  for (int r = 0; r < R; r++) {
    const ksg_profile& prof = profiles[r];
    if (needs_topo(ctx, prof, first, count)) return false;
    int64_t wsum = 0;
    for (int pl : {KSG_PL_NODE_RESOURCES_FIT, KSG_PL_BALANCED_ALLOCATION, KSG_PL_IMAGE_LOCALITY})
      if ((prof.score_mask >> pl) & 1u) {
        if (prof.weight[pl] < 0) return false;
        wsum += prof.weight[pl];
      }
    if (wsum * 100 >= (1ll << 31)) return false;
  }
  for (int i = first; i < first + count; i++)
    if (ctx->h_na_pref_sum[i] > 0xffff || ctx->h_na_pref_sum[i] < 0) return false;
  return true;
}

// mode: 0 generic arithmetic, 1 fast (Fit/BA over {cpu, memory}), 2 fast with
// one scalar Fit column (instantiated for the spill-free shapes only);
// narrow: the 16-byte records (fast modes only)
// MULTI (group barriers): every workgroup must be co-resident; the grid is
// within the occupancy API's residency (run_sweep halves S until it is) and
// the barriers are bounded by a timeout.  A cooperative launch (coop: env
// KSG_COOP_LAUNCH=1, or after a timeout) has the runtime guarantee it.
template <int BLOCK, bool MULTI>
hipError_t launch_one(const void* f, const SweepArgs& s, int grid, hipStream_t st) {
  void* kargs[] = {const_cast<SweepArgs*>(&s)};
  if (MULTI && s.coop) return hipLaunchCooperativeKernel(f, dim3(grid), dim3(BLOCK), kargs, 0, st);
  return hipLaunchKernel(f, dim3(grid), dim3(BLOCK), kargs, 0, st);
}
template <int BLOCK, int KN, bool MULTI>
hipError_t launch_sweep(const SweepArgs& s, int grid, int mode, bool narrow, hipStream_t st) {
  const void* f = mode == 1 && narrow ? (const void*)ksg_sweep<BLOCK, KN, true, MULTI, false, true>
                  : mode == 1 ? (const void*)ksg_sweep<BLOCK, KN, true, MULTI>
                              : (const void*)ksg_sweep<BLOCK, KN, false, MULTI>;
  return launch_one<BLOCK, MULTI>(f, s, grid, st);
}
// The narrow fast sweep of a few replicas over a large cluster with every
// result in registers: 512-lane workgroups at 8 waves per CU (256 VGPRs),
// 64 nodes per lane, so a group of S = N / 32,768 workgroups needs no
// scratch row (configs[4]: S = 4 instead of 8 with the row).
const void* sweep_wide_kernel(int mode) {
  return mode == 2 ? (const void*)ksg_sweep<512, 64, true, true, true, true>
                   : (const void*)ksg_sweep<512, 64, true, true, false, true>;
}

template <int BLOCK, int KN, bool MULTI>
hipError_t launch_sweep_ex(const SweepArgs& s, int grid, bool narrow, hipStream_t st) {
  const void* f = narrow ? (const void*)ksg_sweep<BLOCK, KN, true, MULTI, true, true>
                         : (const void*)ksg_sweep<BLOCK, KN, true, MULTI, true>;
  return launch_one<BLOCK, MULTI>(f, s, grid, st);
}

template <int BLOCK, int KN>
int sweep_occupancy(ksg_ctx* ctx, int mode, bool narrow, int* occ) {   // the MULTI instances
  const void* f = mode == 2 ? (narrow ? (const void*)ksg_sweep<BLOCK, KN, true, true, true, true>
                                      : (const void*)ksg_sweep<BLOCK, KN, true, true, true>)
                  : mode == 1 ? (narrow ? (const void*)ksg_sweep<BLOCK, KN, true, true, false, true>
                                        : (const void*)ksg_sweep<BLOCK, KN, true, true>)
                              : (const void*)ksg_sweep<BLOCK, KN, false, true>;
  HIPC(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, f, BLOCK, 0));
  return KSG_OK;
}

// Host mirror of cm_prof().fast: Fit and BalancedAllocation both score exactly
// {cpu, memory}, Fit with positive weights.
// Host mirror of the sweep's extended fast form (SweepProf::ex): Fit over
// {cpu, memory, one scalar column}, BalancedAllocation over {cpu, memory},
// positive weights.
bool profile_ex_fast(const ksg_profile& prof) {
  if (prof.fit_n != 3 || prof.ba_n != 2 || prof.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO) return false;
  int nc = 0, nm = 0, nx = 0;
  for (int i = 0; i < 3; i++) {
    const int r = prof.fit_res[i];
    nc += r == KSG_RES_CPU;
    nm += r == KSG_RES_MEM;
    nx += r >= 3;
    if (prof.fit_w[i] <= 0) return false;
  }
  const int b0 = prof.ba_res[0], b1 = prof.ba_res[1];
  return nc == 1 && nm == 1 && nx == 1 &&
         ((b0 == KSG_RES_CPU && b1 == KSG_RES_MEM) || (b0 == KSG_RES_MEM && b1 == KSG_RES_CPU));
}

bool profile_cm_fast(const ksg_profile& prof) {
  if (prof.fit_n != 2 || prof.ba_n != 2 || prof.fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO) return false;
  auto cpumem = [](int a, int b) {
    return (a == KSG_RES_CPU && b == KSG_RES_MEM) || (a == KSG_RES_MEM && b == KSG_RES_CPU);
  };
  return cpumem(prof.fit_res[0], prof.fit_res[1]) && cpumem(prof.ba_res[0], prof.ba_res[1]) &&
         prof.fit_w[0] > 0 && prof.fit_w[1] > 0;
}

// The sweep's arithmetic form: 0 generic, 1 fast {cpu, memory}, 2 fast with
// one scalar Fit column.
int sweep_mode(const ksg_profile* profiles, int R) {
  bool fast = true, ex = false;
  for (int r = 0; r < R; r++) {
    const bool cm = profile_cm_fast(profiles[r]), exf = !cm && profile_ex_fast(profiles[r]);
    fast = fast && (cm || exf);
    ex = ex || exf;
  }
  return !fast ? 0 : (ex ? 2 : 1);
}

// Host half of the narrow-state check (the node half is ksg_narrow_init):
// fast arithmetic; every replica filters with Fit and every pod runs it (so
// the Fit filter bounds the requested sums and the pod count); the pods
// request cpu, memory and at most one scalar column, the one every ex
// replica scores (and no replica ignores); memory quantities in whole MiB.
// Fills the pod-side bounds.
bool narrow_candidate(ksg_ctx* ctx, const ksg_profile* profiles, int R, int first, int count, int mode,
                      NarrowBounds* b) {
  if (mode == 0 || ctx->force_path == 3) return false;
  int nx = -1;
  for (int r = 0; r < R; r++) {
    const ksg_profile& prof = profiles[r];
    bool fit = false;
    for (int k = 0; k < prof.n_filter; k++) fit |= prof.filter_order[k] == KSG_PL_NODE_RESOURCES_FIT;
    if (!fit) return false;
    int64_t fw = 0;   // Fit's weighted score numerator stays below 2^30 (sweep_cm_scores32)
    for (int i = 0; i < prof.fit_n; i++) fw += prof.fit_w[i] > 0 ? prof.fit_w[i] : 0;
    if (fw * 100 >= (1 << 30)) return false;
    if (mode == 2 && !profile_cm_fast(prof))
      for (int i = 0; i < prof.fit_n; i++)
        if (prof.fit_res[i] >= 3) {
          if (nx >= 0 && nx != prof.fit_res[i]) return false;
          nx = prof.fit_res[i];
        }
  }
  if (mode == 2 && nx < 0) return false;
  for (int r = 0; r < R; r++)
    if (nx >= 0 && ((profiles[r].fit_ignored_res >> nx) & 1u)) return false;
  constexpr int64_t kMiB = (int64_t)1 << kNarrowMemShift;
  int64_t xc = 0, xm = 0;
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if ((p.filter_skip >> KSG_PL_NODE_RESOURCES_FIT) & 1u) return false;
    for (int r = 0; r < KSG_MAX_RES; r++)
      if (p.req[r] < 0 || (r >= 2 && r != nx && p.req[r] != 0)) return false;
    if (p.req[KSG_RES_CPU] > INT32_MAX || p.nz_cpu < 0 || p.nz_cpu > INT32_MAX) return false;
    if (nx >= 0 && p.req[nx] > 255) return false;
    if (((p.req[KSG_RES_MEM] | p.nz_mem) & (kMiB - 1)) != 0 || p.nz_mem < 0) return false;
    if ((p.req[KSG_RES_MEM] >> kNarrowMemShift) > INT32_MAX) return false;
    xc = std::max(xc, p.nz_cpu - p.req[KSG_RES_CPU]);
    xm = std::max(xm, (p.nz_mem - p.req[KSG_RES_MEM]) >> kNarrowMemShift);
  }
  if (xc > INT32_MAX || xm >= ((int64_t)1 << 24)) return false;
  b->xc = xc;
  b->xm = xm;
  b->nx = nx;
  b->places = std::min(count, 255);
  return true;
}

// R replicas of pods [first, first + count) on the state already copied into
// a.st (replica strides set), or on the narrow records when nstat is set;
// placements [R][count] on the device.
int run_sweep(ksg_ctx* ctx, const QueueArgs& a, const ksg_profile* profiles, const ksg_profile* d_prof, int R,
              int first, int count, int32_t* d_pl, Tmp& tmp, const int4* nstat = nullptr,
              const double2* nrcp = nullptr, int4* nmut = nullptr, int nx = -1) {
  const int mode = sweep_mode(profiles, R);
  const bool narrow = nstat != nullptr;
  const int N = ctx->c.N;
  constexpr int kBatch = 64;
  SweepArgs s{};
  s.c = ctx->c;
  s.st = a.st;
  s.pods = ctx->d_pods;
  s.prog = ctx->d_prog;
  s.profiles = d_prof;
  s.count = count;
  s.placements = d_pl;
  s.nstat = nstat;
  s.nrcp = nrcp;   // DevCluster::rcp64 on the narrow path
  s.nmut = nmut;
  s.nx = nx;
  s.coop = ctx->coop_launch ? 1 : 0;
  TA(tmp, &s.srec, sizeof(uint64_t) * (size_t)kBatch * N);
  // Workgroups per replica: with few replicas of a large cluster, S > 1 spreads
  // each replica over S co-resident workgroups (two group barriers per pod);
  // aim at ~2 workgroups per CU and at least ~8 nodes per lane (config 5,
  // 64 replicas x 100k nodes: S = 8 runs 5 % faster than S = 16 and 1.2x
  // faster than S = 4; profiles/r1/config5_group_size.json).
  int cus = 0;
  HIPC(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
  int S = 1;
  if (R < 2 * cus) S = std::min({std::max(1, 2 * cus / R), std::max(1, N / 2048), 64});
  // Measurement knob: force the group size (still halved below until every
  // workgroup of a group is co-resident, so a forced S cannot deadlock).
  if (const char* f = getenv("KSG_SWEEP_S")) S = std::max(1, std::min(atoi(f), 64));
  // (BLOCK, KN): KN nodes per lane in registers; KN = 0 streams them through a
  // per-replica scratch row instead.  The instances that fit 128 VGPRs without
  // spilling: every fast shape for one workgroup per replica; KN = 8 for
  // several (runtime stride) and for the generic arithmetic.
  struct Shape { int block, kn; };
  static const Shape fast1[] = {{256, 8}, {256, 16}, {256, 20}, {256, 24}, {256, 32}, {512, 32}, {1024, 32}};
  static const Shape fastm[] = {{256, 8}};
  static const Shape gen[] = {{256, 8}};
  int block = 1024, kn = 0;
  for (;;) {
    const int neff = (N + S - 1) / S;
    const Shape* list = mode == 1 ? (S == 1 ? fast1 : fastm) : gen;
    const int nl = mode == 1 && S == 1 ? 7 : 1;
    block = S > 1 || neff <= 16384 ? 256 : 1024;
    kn = 0;
    for (int i = 0; i < nl; i++)
      if (neff <= list[i].block * list[i].kn) { block = list[i].block; kn = list[i].kn; break; }
    if (S == 1) break;
    int occ = 0, rc0 = 0;
    switch (block * 100 + kn) {
      case 25608: rc0 = sweep_occupancy<256, 8>(ctx, mode, narrow, &occ); break;
      default: rc0 = sweep_occupancy<256, 0>(ctx, mode, narrow, &occ); break;
    }
    if (rc0) return rc0;
    if ((long long)R * S <= (long long)occ * cus) break;   // every workgroup of a group co-resident
    S = S / 2;
  }
  // the register-resident wide form when the scratch form was chosen for the
  // narrow fast state and its groups are co-resident
  bool wide = false;
  if (kn == 0 && S > 1 && mode >= 1 && narrow && !getenv("KSG_SWEEP_NO_WIDE")) {
    const int S2 = (N + 512 * 64 - 1) / (512 * 64);
    int occ = 0;
    HIPC(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, sweep_wide_kernel(mode), 512, 0));
    if (S2 > 1 && (long long)R * S2 <= (long long)occ * cus) {
      wide = true;
      S = S2;
      block = 512;
      kn = 64;
    }
  }
  s.S = S;
  if (kn == 0) TA(tmp, &s.scratch, sizeof(uint64_t) * (size_t)R * N);
  if (S > 1) {
    TA(tmp, &s.slots, sizeof(SweepSlot) * 2 * (size_t)R * S);
    TA(tmp, &s.gbar, sizeof(unsigned) * 16 * (size_t)R);
    TA(tmp, &s.timeout, 16);
    HIPC(ctx, hipMemsetAsync(s.timeout, 0, 16, ctx->stream));
    if ((ctx->inject_timeout & 4) && !s.coop) {   // test injection: the group barriers find it set
      ctx->inject_timeout &= ~4;
      HIPC(ctx, hipMemsetAsync(s.timeout, 0x01, sizeof(unsigned), ctx->stream));
    }
  }
  (void)hipGetLastError();
  treset(ctx);
  HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  int rc;
  if ((rc = tmark(ctx))) return rc;
  for (int off = 0; off < count; off += kBatch) {
    s.b0 = first + off;
    s.nb = std::min(kBatch, count - off);
    s.out0 = off;
    hipLaunchKernelGGL(ksg_sweep_static, dim3(static_blocks(N, s.nb)), dim3(256), 0, ctx->stream, s);
    if ((rc = tlaunched(ctx, KSG_K_SWEEP_STATIC, (double)s.nb * N))) return rc;
    if (S > 1) HIPC(ctx, hipMemsetAsync(s.gbar, 0, sizeof(unsigned) * 16 * (size_t)R, ctx->stream));
    const int grid = R * S;
    const int key = block * 100 + kn;
    hipError_t le;
    if (wide) {
      le = launch_one<512, true>(sweep_wide_kernel(mode), s, grid, ctx->stream);
    } else if (mode == 2) {
      if (S > 1) {
        if (key == 25608) le = launch_sweep_ex<256, 8, true>(s, grid, narrow, ctx->stream);
        else le = launch_sweep_ex<256, 0, true>(s, grid, narrow, ctx->stream);
      } else {
        if (key == 25608) le = launch_sweep_ex<256, 8, false>(s, grid, narrow, ctx->stream);
        else if (key == 25600) le = launch_sweep_ex<256, 0, false>(s, grid, narrow, ctx->stream);
        else le = launch_sweep_ex<1024, 0, false>(s, grid, narrow, ctx->stream);
      }
    } else if (S > 1) {
      switch (key) {
        case 25608: le = launch_sweep<256, 8, true>(s, grid, mode, narrow, ctx->stream); break;
        default: le = launch_sweep<256, 0, true>(s, grid, mode, narrow, ctx->stream); break;
      }
    } else {
      switch (key) {
        case 25608: le = launch_sweep<256, 8, false>(s, grid, mode, narrow, ctx->stream); break;
        case 25616: le = launch_sweep<256, 16, false>(s, grid, mode, narrow, ctx->stream); break;
        case 25620: le = launch_sweep<256, 20, false>(s, grid, mode, narrow, ctx->stream); break;
        case 25624: le = launch_sweep<256, 24, false>(s, grid, mode, narrow, ctx->stream); break;
        case 25632: le = launch_sweep<256, 32, false>(s, grid, mode, narrow, ctx->stream); break;
        case 51232: le = launch_sweep<512, 32, false>(s, grid, mode, narrow, ctx->stream); break;
        case 102432: le = launch_sweep<1024, 32, false>(s, grid, mode, narrow, ctx->stream); break;
        case 25600: le = launch_sweep<256, 0, false>(s, grid, mode, narrow, ctx->stream); break;
        default: le = launch_sweep<1024, 0, false>(s, grid, mode, narrow, ctx->stream); break;
      }
    }
    HIPC(ctx, le);
    if ((rc = tlaunched(ctx, narrow ? KSG_K_SWEEP_NARROW : KSG_K_SWEEP, (double)R * s.nb * N))) return rc;
  }
  ctx->sweep_timeout = S > 1 ? s.timeout : nullptr;
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  return KSG_OK;
}

// Single replica, PodTopologySpread / InterPodAffinity, no capture: the queue
// on G co-resident workgroups (ksched_topo_coop.h), in batches of kCoopBatch
// pods, each preceded by its static records (ksg_sweep_static).
template <int KN, bool LL = false>
int coop_occupancy(ksg_ctx* ctx, int* occ) {
  HIPC(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, (const void*)ksg_topo_coop<KN, LL>, 256, 0));
  return KSG_OK;
}

// The capture outputs of a chip-wide topology run (CoopArgs cap_*; mode 1
// device rows of a captured queue, mode 2 the per-cycle host block).
struct CoopCap {
  int mode = 0;
  uint32_t* fs = nullptr;
  char *raw = nullptr, *norm = nullptr, *tot = nullptr;
  int32_t rows[KSG_NPLUGINS] = {};
  int32_t n_rows = 0, n_normrows = 0, narrow = 0;
  int32_t es = 8;                     // mode 2: bytes per row value
  ksg_result* h_res = nullptr;
  unsigned* h_flag = nullptr;
  unsigned* h_ovf = nullptr;
  unsigned seq = 0;
  // mode 2, the pod's append still staged: read from the staging buffer (its
  // device address) and copied to the device pool by workgroup 0
  const char* stage = nullptr;
  int64_t stage_base = 0, stage_len = 0;
};

// ksg_topo_coop<KN, LL, CAP>: capture instances exist for KN <= 4 (up to
// 262,144 nodes); nullptr where there is none.
const void* coop_kernel(int kn, bool ll, int cap) {
  if (cap == 0)
    return ll ? (const void*)ksg_topo_coop<1, true> : kn == 1 ? (const void*)ksg_topo_coop<1> : kn == 2 ? (const void*)ksg_topo_coop<2>
         : kn == 4 ? (const void*)ksg_topo_coop<4> : kn == 8 ? (const void*)ksg_topo_coop<8>
         : kn == 16 ? (const void*)ksg_topo_coop<16> : (const void*)ksg_topo_coop<32>;
  if (cap == 1)
    return ll ? (const void*)ksg_topo_coop<1, true, 1> : kn == 1 ? (const void*)ksg_topo_coop<1, false, 1>
         : kn == 2 ? (const void*)ksg_topo_coop<2, false, 1> : kn == 4 ? (const void*)ksg_topo_coop<4, false, 1> : nullptr;
  return ll ? (const void*)ksg_topo_coop<1, true, 2> : kn == 1 ? (const void*)ksg_topo_coop<1, false, 2>
       : kn == 2 ? (const void*)ksg_topo_coop<2, false, 2> : kn == 4 ? (const void*)ksg_topo_coop<4, false, 2> : nullptr;
}

// The maintained domain tables for a topology run of pods [first, first +
// count): the (selector, non-unique column) pairs, the unique-key hard
// selectors and the totals their programs read (the same program layout as
// parse_topo), laid out in one device block and rebuilt from cnt and the
// labels by ksg_topo_tables_init.  Returns false (tables unused) when the
// layout would not fit its limits.
// universe: every (selector, non-unique column) pair and every selector's
// count-of-counts, no per-pod scope (the per-cycle tables: the topology
// kernel computes each pod's scope itself, tables_fill), into ctx->d_pct.
bool build_topo_tables(ksg_ctx* ctx, int32_t first, int32_t count, TopoTables* out, int* rc,
                       bool universe = false) {
  *rc = KSG_OK;
  const int S = ctx->c.S, L = ctx->c.L, N = ctx->c.N;
  if (S <= 0 || L <= 0 || (size_t)S * L > (1u << 24)) return false;
  constexpr int kKc = 256;   // count-of-counts bins: a node's matching pods stay below 255
  std::vector<int32_t> pair_off((size_t)S * L, -1), cc_off(S, -1), pres_off(L, -1);
  std::vector<uint8_t> want_tot(S, 0);
  std::vector<TopoTableTask> tasks;
  size_t dom_words = 0, cc_words = 0, pres_words = 0;
  bool fits = true;
  auto pair = [&](int sel, int col) {
    if (sel < 0 || col < 0 || col >= L || ctx->h_col_unique[col] || sel >= S) return;
    const int V = ctx->h_col_vocab[col];
    if (V > kTableLds) { fits = false; return; }
    int32_t& o = pair_off[(size_t)sel * L + col];
    if (o >= 0) return;
    o = (int32_t)dom_words;
    int po = -1;
    if (pres_off[col] < 0) {
      pres_off[col] = (int32_t)pres_words;
      po = pres_off[col];
      pres_words += (V + 31) / 32;
    }
    tasks.push_back(TopoTableTask{0, sel, col, o, po});
    dom_words += V;
  };
  auto cc = [&](int sel) {
    if (sel < 0 || sel >= S || cc_off[sel] >= 0) return;
    cc_off[sel] = (int32_t)cc_words;
    cc_words += kKc;
    want_tot[sel] = 1;
  };
  const int32_t* P = ctx->h_prog.data();
  if (universe) {
    count = 0;
    bool any_unique = false;
    for (int col = 0; col < L; col++) any_unique = any_unique || ctx->h_col_unique[col];
    for (int sel = 0; sel < S; sel++) {
      for (int col = 0; col < L; col++)
        if (!ctx->h_col_unique[col]) pair(sel, col);
      if (any_unique) cc(sel);
      want_tot[sel] = 1;
    }
  }
  for (int i = first; i < first + count; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    if (p.pts >= 0) {
      const int32_t* w = P + p.pts;
      const int nh = w[0], ns = w[1];
      const int32_t* hard = w + 3;
      for (int k = 0; k < nh; k++) {
        const int col = hard[7 * k], sel = hard[7 * k + 1];
        if (col >= 0 && col < L && ctx->h_col_unique[col]) cc(sel);
        else pair(sel, col);
      }
      const int32_t* soft = hard + 7 * nh;
      for (int k = 0; k < ns; k++)
        if (!soft[6 * k + 5]) pair(soft[6 * k + 1], soft[6 * k]);
    }
    if (p.ipa >= 0) {
      const int32_t* w = P + p.ipa;
      const int na = w[0], sel_all = w[1];
      for (int k = 0; k < na; k++) {
        const int col = w[3 + k];
        if (col >= 0 && col < L && ctx->h_col_unique[col]) { if (sel_all >= 0 && sel_all < S) want_tot[sel_all] = 1; }
        else pair(sel_all, col);
      }
      w += 3 + na;
      const int nanti = *w++;
      for (int k = 0; k < nanti; k++) pair(w[2 * k + 1], w[2 * k]);
      w += 2 * nanti;
      const int npref = *w++;
      for (int k = 0; k < npref; k++) {
        const int col = w[3 * k], sel = w[3 * k + 1];
        if (col >= 0 && col < L && ctx->h_col_unique[col]) { if (sel >= 0 && sel < S) want_tot[sel] = 1; }
        else pair(sel, col);
      }
    }
  }
  if (!fits || dom_words > (64u << 20)) return false;
  for (int s = 0; s < S; s++)
    if (want_tot[s]) tasks.push_back(TopoTableTask{1, s, 0, cc_off[s], -1});
  for (int col = 0; col < L; col++) tasks.push_back(TopoTableTask{2, 0, col, 0, -1});
  // each selector's (column, table offset) pairs (lag_apply)
  std::vector<int32_t> sp_off(S + 1, 0), sp;
  for (int s = 0; s < S; s++) {
    sp_off[s] = (int32_t)(sp.size() / 2);
    for (int col = 0; col < L; col++) {
      const int32_t o = pair_off[(size_t)s * L + col];
      if (o >= 0) { sp.push_back(col); sp.push_back(o); }
    }
  }
  sp_off[S] = (int32_t)(sp.size() / 2);
  // block: dom | tot[S] | cc | pres | col_missing[L] | col_empty[L] | invalid | pair_off[S*L] | cc_off[S] |
  // pres_off[L] | sp_off[S+1] | sp | elig[count] (bytes) | fill tasks [count][kTopoFill] int4 | tasks
  const size_t o_tot = dom_words, o_cc = o_tot + S, o_pres = o_cc + cc_words, o_miss = o_pres + pres_words,
               o_empty = o_miss + L, o_inv = o_empty + L, o_pair = o_inv + 1, o_ccoff = o_pair + (size_t)S * L,
               o_preso = o_ccoff + S, o_spoff = o_preso + L, o_sp = o_spoff + S + 1, o_elig = o_sp + sp.size(),
               o_fo = (o_elig + ((size_t)count + 3) / 4 + 3) & ~(size_t)3,
               o_tasks = o_fo + (size_t)count * kTopoFill * 4,
               words = o_tasks + tasks.size() * (sizeof(TopoTableTask) / 4);
  int32_t*& buf = universe ? ctx->d_pct : ctx->d_tables;
  size_t& buf_words = universe ? ctx->pct_words : ctx->tables_words;
  if (words > buf_words) {
    if (buf) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)buf);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) { *rc = fail(ctx, KSG_E_DEVICE, "tables: sync"); return false; }
      (void)hipFree(buf);
      buf = nullptr;
      buf_words = 0;
    }
    if ((*rc = dalloc(ctx, &buf, words))) return false;
    buf_words = words;
  }
  int32_t* b = buf;
  auto up = [&](size_t off, const void* src, size_t bytes) {
    return hipMemcpyAsync(b + off, src, bytes, hipMemcpyHostToDevice, ctx->stream) == hipSuccess;
  };
  bool ok = hipMemsetAsync(b, 0, sizeof(int32_t) * o_pair, ctx->stream) == hipSuccess &&
            up(o_pair, pair_off.data(), sizeof(int32_t) * pair_off.size()) &&
            up(o_ccoff, cc_off.data(), sizeof(int32_t) * S) && up(o_preso, pres_off.data(), sizeof(int32_t) * L) &&
            up(o_spoff, sp_off.data(), sizeof(int32_t) * (S + 1)) &&
            (sp.empty() || up(o_sp, sp.data(), sizeof(int32_t) * sp.size())) &&
            up(o_tasks, tasks.data(), sizeof(TopoTableTask) * tasks.size());
  if (!ok) { *rc = fail(ctx, KSG_E_DEVICE, "tables: upload"); return false; }
  TopoTables t{};
  t.dom = b;
  t.tot = b + o_tot;
  t.cc = b + o_cc;
  t.pair_off = b + o_pair;
  t.cc_off = b + o_ccoff;
  t.pres = reinterpret_cast<uint32_t*>(b + o_pres);
  t.pres_off = b + o_preso;
  t.col_missing = b + o_miss;
  t.col_empty = b + o_empty;
  t.invalid = reinterpret_cast<unsigned*>(b + o_inv);
  t.sp_off = b + o_spoff;
  t.sp = b + o_sp;
  t.elig = reinterpret_cast<const uint8_t*>(b + o_elig);
  t.fo = reinterpret_cast<const int4*>(b + o_fo);
  t.first = first;
  t.S = S;
  t.L = L;
  t.Kc = kKc;
  hipLaunchKernelGGL(ksg_topo_tables_init, dim3((unsigned)tasks.size()), dim3(256), 0, ctx->stream, ctx->c, ctx->st,
                     t, reinterpret_cast<const TopoTableTask*>(b + o_tasks));
  if (hipGetLastError() != hipSuccess) { *rc = fail(ctx, KSG_E_DEVICE, "tables: init launch"); return false; }
  if (count > 0) {
    hipLaunchKernelGGL(ksg_topo_tables_elig, dim3((unsigned)((count + 63) / 64)), dim3(64), 0, ctx->stream, ctx->c, t,
                       ctx->d_pods, ctx->d_prog, count, reinterpret_cast<uint8_t*>(b + o_elig),
                       reinterpret_cast<int4*>(b + o_fo));
    if (hipGetLastError() != hipSuccess) { *rc = fail(ctx, KSG_E_DEVICE, "tables: scope launch"); return false; }
  }
  (void)N;
  *out = t;
  return true;
}

// The chip-wide topology path's group shape (nodes per lane, G, the LDS
// variant), once per node set.
int coop_shape(ksg_ctx* ctx) {
  const int N = ctx->c.N;
  int rc;
  if (ctx->coop_cfg_N != N) {   // the group shape, once per node set
    int cus = 0;
    HIPC(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    if (!ctx->coop_gmax) ctx->coop_gmax = std::min(cus, 256);   // one workgroup per CU: lanes wait on memory
    int kn = 1;
    while ((size_t)kn * 256 * ctx->coop_gmax < (size_t)N && kn < 32) kn *= 2;
    if ((size_t)kn * 256 * ctx->coop_gmax < (size_t)N) return fail(ctx, KSG_E_UNSUPPORTED, "topology path: too many nodes");
    const int G = (int)((N + 256 * kn - 1) / (256 * kn));
    // the variant whose label / vocabulary / template tables are LDS at compile time
    const bool ll = kn == 1 && ctx->c.L <= kCoopLabCols && ctx->c.n_tmpl <= kCoopTmpl;
    int occ = 0;
    switch (kn) {
      case 1: rc = ll ? coop_occupancy<1, true>(ctx, &occ) : coop_occupancy<1>(ctx, &occ); break;
      case 2: rc = coop_occupancy<2>(ctx, &occ); break;
      case 4: rc = coop_occupancy<4>(ctx, &occ); break;
      case 8: rc = coop_occupancy<8>(ctx, &occ); break;
      case 16: rc = coop_occupancy<16>(ctx, &occ); break;
      default: rc = coop_occupancy<32>(ctx, &occ); break;
    }
    if (rc) return rc;
    if (G > occ * cus) return fail(ctx, KSG_E_UNSUPPORTED, "topology path: grid exceeds co-resident workgroups");
    ctx->coop_kn = kn;
    ctx->coop_G = G;
    ctx->coop_ll = ll;
    ctx->coop_cfg_N = N;
    ctx->coop_dirty = true;   // (the one-pod completion counter counts arrivals modulo G)
  }
  return KSG_OK;
}

int run_topo_coop(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* d_pl, ksg_result* d_res,
                  const ksg_profile* d_prof, int do_commit = 1, const CoopCap* cap = nullptr,
                  bool timed = true) {
  const int N = ctx->c.N;
  int rc;
  if ((rc = coop_shape(ctx))) return rc;
  const int kn = ctx->coop_kn, G = ctx->coop_G;
  const bool ll = ctx->coop_ll;
  if (!ctx->d_coop_acc) {
    if ((rc = dalloc(ctx, &ctx->d_coop_acc, 2))) return rc;
    if (!ctx->d_coop_flags && (rc = dalloc(ctx, &ctx->d_coop_flags, 8))) return rc;   // [4] timeout, [6] one-pod
                                                                                      // completion counter
    if ((rc = dalloc(ctx, &ctx->d_coop_wgflags, (size_t)256 * 32))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_coop_parts, 256))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_coop_phist, (size_t)256 * kCoopPHist))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_coop_srec, (size_t)kCoopBatch * N))) return rc;
    ctx->coop_dirty = true;
  }
  // the barrier flags are monotonic across launches ((gen << 16) + epoch, a
  // launch runs < 2^16 barriers); reset with the atomics sets and the timeout
  // word after a failed launch or when the generation wraps
  const int n_launch = (count + kCoopBatch - 1) / kCoopBatch;
  if (ctx->coop_dirty || ctx->coop_gen + (unsigned)n_launch >= 0xffffu) {
    HIPC(ctx, hipMemsetAsync(ctx->d_coop_wgflags, 0, sizeof(unsigned) * 32 * 256, ctx->stream));
    HIPC(ctx, hipMemsetAsync(ctx->d_coop_acc, 0, 2 * sizeof(CoopAcc), ctx->stream));
    HIPC(ctx, hipMemsetAsync(ctx->d_coop_flags, 0, 32, ctx->stream));
    ctx->coop_gen = 0;
    ctx->coop_dirty = false;
  }
  CoopArgs a{};
  a.c = ctx->c;
  a.st = ctx->st;
  a.pods = ctx->d_pods;
  a.prog = ctx->d_prog;
  a.profile = d_prof;
  a.G = G;
  a.placements = d_pl;
  a.results = d_res;
  a.srec = ctx->d_coop_srec;
  a.parts = ctx->d_coop_parts;
  a.phist = ctx->d_coop_phist;
  a.acc = ctx->d_coop_acc;
  a.bar = ctx->d_coop_wgflags;
  a.pmode = ctx->coop_pmode;
  a.timeout = ctx->d_coop_flags + 4;
  a.arrive = ctx->d_coop_flags + 6;
  a.commit = do_commit;
  // the maintained tables: placement runs (they are rebuilt per run from the
  // state; a single-pod evaluation runs phase 1 instead of paying the rebuild)
  if (ctx->coop_tables && do_commit && count > 1) {
    ctx->pct_valid = false;   // the run moves the counts without the per-cycle tables
    TopoTables t{};
    if (build_topo_tables(ctx, first, count, &t, &rc)) {
      a.tt = t;
      a.use_tables = 1;
    } else if (rc) {
      return rc;
    }
  } else if (ctx->coop_tables && ctx->pc_tables && !do_commit && count == 1 && cap && cap->mode == 2) {
    // the per-cycle evaluation: the universe's tables, built once per
    // encoding and kept exact by every ksg_commit / ksg_uncommit since
    if (!ctx->pct_valid) {
      TopoTables t{};
      if (build_topo_tables(ctx, 0, 0, &t, &rc, true)) {
        ctx->pct = t;
        ctx->pct_valid = true;
      } else if (rc) {
        return rc;
      } else {
        ctx->pc_tables = false;   // the layout does not fit its limits: the pre-pass from now on
      }
    }
    if (ctx->pct_valid) {
      a.tt = ctx->pct;
      a.use_tables = 1;
      a.tables_inkernel = 1;
    }
  } else if (do_commit) {
    ctx->pct_valid = false;
  }
  if (!a.use_tables) {   // the kernel reads tt.invalid and the index arrays at setup: a valid empty set
    if (!ctx->d_coop_notables) {
      if ((rc = dalloc(ctx, &ctx->d_coop_notables, 64))) return rc;
      HIPC(ctx, hipMemsetAsync(ctx->d_coop_notables, 0, 64 * sizeof(int32_t), ctx->stream));
    }
    TopoTables t{};
    t.invalid = reinterpret_cast<unsigned*>(ctx->d_coop_notables);
    a.tt = t;
  }
  const int cmode = cap ? cap->mode : 0;
  const void* kf = coop_kernel(kn, ll, cmode);
  if (!kf) return fail(ctx, KSG_E_UNSUPPORTED, "topology path: no capture instance for this many nodes");
  if (cap) {
    a.cap_fs = cap->fs;
    a.cap_raw = cap->raw;
    a.cap_norm = cap->norm;
    a.cap_tot = cap->tot;
    for (int q = 0; q < KSG_NPLUGINS; q++) a.cap_rows[q] = cap->rows[q];
    a.cap_n_rows = cap->n_rows;
    a.cap_n_normrows = cap->n_normrows;
    a.cap_narrow = cap->narrow;
    a.cap_es = cap->es;
    a.h_res = cap->h_res;
    a.h_flag = cap->h_flag;
    a.h_ovf = cap->h_ovf;
    a.seq = cap->seq;
    if (cap->stage) {   // pods + first and prog + blob address the staged record and programs
      const int32_t* sprog = reinterpret_cast<const int32_t*>(cap->stage + sizeof(ksg_pod));
      a.pods = reinterpret_cast<const ksg_pod*>(cap->stage) - first;
      a.prog = sprog - cap->stage_base;
      a.wpods = ctx->d_pods + first;
      a.wprog = ctx->d_prog + cap->stage_base;
      a.sprog = sprog;
      a.slen = cap->stage_len;
    }
  }
  // one pod evaluated (the per-cycle path): the static records in place, a
  // plain launch (every workgroup one per CU, the barrier's poll is bounded;
  // the caller relaunches cooperatively if they were not all resident)
  const bool one = count == 1 && cmode == 2;
  a.fused_static = one ? 1 : 0;
  SweepArgs sa{};
  sa.c = ctx->c;
  sa.pods = ctx->d_pods;
  sa.prog = ctx->d_prog;
  sa.profiles = d_prof;
  sa.srec = ctx->d_coop_srec;
#ifdef KSG_STAMPS
  if (!ctx->d_stamps) {
    if ((rc = dalloc(ctx, &ctx->d_stamps, 16))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_stamps, 0, 128, ctx->stream));
  }
  a.stamps = ctx->d_stamps;
#endif
  (void)hipGetLastError();
  treset(ctx);
  if (timed) HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  if ((rc = tmark(ctx))) return rc;
  for (int off = 0; off < count; off += kCoopBatch) {
    const int nb = std::min(kCoopBatch, count - off);
    sa.b0 = first + off;
    sa.nb = nb;
    if (cap && cap->mode == 1) {   // this launch's pods start at row `off` of the capture arrays
      const size_t es = cap->narrow ? 4 : 8, NN = N;
      a.cap_fs = cap->fs + (size_t)off * NN;
      a.cap_raw = cap->raw + (size_t)off * cap->n_rows * NN * es;
      a.cap_norm = cap->norm + (size_t)off * cap->n_normrows * NN * es;
      a.cap_tot = cap->tot + (size_t)off * NN * es;
    }
    if (!one) {
      hipLaunchKernelGGL(ksg_sweep_static, dim3(static_blocks(N, nb)), dim3(256), 0, ctx->stream, sa);
      if ((rc = tlaunched(ctx, KSG_K_SWEEP_STATIC, (double)nb * N))) return rc;
    }
    a.first = first + off;
    a.count = nb;
    a.out0 = off;
    a.gen = ++ctx->coop_gen;
    {   // test injection: the barriers of this launch (the second of a queue
        // run, so the first 64 pods are committed) find the timeout word set
      const int bit = one ? 2 : 1;
      if ((ctx->inject_timeout & bit) && !(one ? ctx->topo_eval_coop : ctx->coop_launch) &&
          off == (count > kCoopBatch ? kCoopBatch : 0)) {
        ctx->inject_timeout &= ~bit;
        HIPC(ctx, hipMemsetAsync(ctx->d_coop_flags + 4, 0x01, sizeof(unsigned), ctx->stream));
      }
    }
    // the grid barrier needs the G workgroups co-resident: G is within the
    // occupancy API's residency; a cooperative launch (ctx->coop_launch, or
    // the one-pod evaluation after a timeout) has the runtime guarantee it
    void* kargs[] = {&a};
    if (one ? !ctx->topo_eval_coop : !ctx->coop_launch)
      HIPC(ctx, hipLaunchKernel(kf, dim3(G), dim3(256), kargs, 0, ctx->stream));
    else
      HIPC(ctx, hipLaunchCooperativeKernel(kf, dim3(G), dim3(256), kargs, 0, ctx->stream));
    if ((rc = tlaunched(ctx, KSG_K_TOPO_COOP, (double)nb * N))) return rc;
  }
  HIPC(ctx, hipGetLastError());
  if (timed) HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  return KSG_OK;
}

// The speculative topology queue (ksched_topo_win.h) over pods [first, first +
// count) of a placement run.  *used = false (nothing launched) when the run is
// outside its scope: one node per lane, no host ports or volumes (an assume
// that changes what a node-local plugin reads outside the walk's
// re-evaluation), the maintained tables, at least two rows of G workgroups
// co-resident; the caller then runs ksg_topo_coop.
//
// Window lengths come from the pods' programs alone: pod j joins the window
// of the pods before it when none of them writes (commit program: matched
// selectors, owned templates) what j reads (its constraints' and terms'
// selectors, the templates matching it).  The launches are device-driven: the
// host enqueues one (rows, walk) pair per window the lengths predict, then
// reads the cursor once; a window the walk ended early leaves pods for a
// second, shorter round.
int run_topo_window(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* d_pl, ksg_result* d_res,
                    const ksg_profile* d_prof, bool* used) {
  *used = false;
  int rc;
  if (!ctx->topo_window || ctx->coop_launch || !ctx->coop_tables || count < 2) return KSG_OK;
  if ((rc = coop_shape(ctx))) return rc;
  if (ctx->coop_kn != 1) return KSG_OK;
  for (int32_t i = first; i < first + count; i++)
    if (ctx->h_pods[i].ports >= 0 || ctx->h_pods[i].vol >= 0) return KSG_OK;
  const int N = ctx->c.N, G = ctx->coop_G;
  const bool ll = ctx->coop_ll;
  const void* kf = ll ? (const void*)ksg_topo_coop<1, true, 3> : (const void*)ksg_topo_coop<1, false, 3>;
  int occ = 0, cus = 0;
  HIPC(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kf, 256, 0));
  HIPC(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
  const int kmax = std::min(ctx->win_kmax, (occ * cus) / std::max(G, 1));
  if (kmax < 2) return KSG_OK;
  TopoTables tt{};
  if (!build_topo_tables(ctx, first, count, &tt, &rc)) return rc;
  ctx->pct_valid = false;   // the run moves the counts without the per-cycle tables
  // ---- window lengths -------------------------------------------------------
  const int S = ctx->c.S, T = ctx->c.n_tmpl;
  const int32_t* P = ctx->h_prog.data();
  std::vector<int32_t> rd_off(count + 1, 0), wr_off(count + 1, 0), rd, wr;
  for (int32_t k = 0; k < count; k++) {
    const ksg_pod& p = ctx->h_pods[first + k];
    auto sel = [&](std::vector<int32_t>& v, int32_t s) { if (s >= 0 && s < S) v.push_back(s); };
    auto tmpl = [&](std::vector<int32_t>& v, int32_t t) { if (t >= 0 && t < T) v.push_back(S + t); };
    if (p.pts >= 0) {
      const int32_t* w = P + p.pts;
      const int nh = w[0], ns = w[1];
      for (int q = 0; q < nh; q++) sel(rd, w[3 + 7 * q + 1]);
      for (int q = 0; q < ns; q++) sel(rd, w[3 + 7 * nh + 6 * q + 1]);
    }
    if (p.ipa >= 0) {
      const int32_t* w = P + p.ipa;
      const int na = w[0];
      if (na > 0) sel(rd, w[1]);
      w += 3 + na;
      const int nanti = *w++;
      for (int q = 0; q < nanti; q++) sel(rd, w[2 * q + 1]);
      w += 2 * nanti;
      const int npref = *w++;
      for (int q = 0; q < npref; q++) sel(rd, w[3 * q + 1]);
      w += 3 * npref;
      for (int lst = 0; lst < 3; lst++) {
        const int nm = *w++;
        for (int q = 0; q < nm; q++) tmpl(rd, w[q]);
        w += nm;
      }
    }
    if (p.commit >= 0) {
      const int32_t* w = P + p.commit;
      const int ns = w[0];
      for (int q = 0; q < ns; q++) sel(wr, w[1 + q]);
      const int nt = w[1 + ns];
      for (int q = 0; q < nt; q++) tmpl(wr, w[2 + ns + 2 * q]);
    }
    rd_off[k + 1] = (int32_t)rd.size();
    wr_off[k + 1] = (int32_t)wr.size();
  }
  std::vector<int32_t> wlen(count), stamp((size_t)S + T, -1);
  for (int32_t s0 = 0; s0 < count; s0++) {
    int len = 0;
    for (int32_t j = s0; j < count && len < kmax; j++, len++) {
      bool clash = false;
      for (int32_t q = rd_off[j]; q < rd_off[j + 1] && !clash; q++) clash = stamp[rd[q]] == s0;
      if (clash) break;
      for (int32_t q = wr_off[j]; q < wr_off[j + 1]; q++) stamp[wr[q]] = s0;
    }
    wlen[s0] = std::max(len, 1);
  }
  auto windows_from = [&](int32_t pos) {   // launches if no window ends early
    int n = 0;
    while (pos < count) { pos += wlen[pos]; n++; }
    return n;
  };
  // ---- the device block ------------------------------------------------------
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_cur = 0, o_stats = 128, o_len = 256, o_tot = o_len + al(sizeof(int32_t) * count),
               o_top = o_tot + al(sizeof(int32_t) * kmax * N),
               o_pod = o_top + al(sizeof(unsigned long long) * kmax * G * kmax),
               o_parts = o_pod + al(sizeof(WinPod) * kmax), o_phist = o_parts + al(sizeof(CoopPart) * kmax * G),
               o_acc = o_phist + al(sizeof(int32_t) * kmax * G * kCoopPHist),
               o_bar = o_acc + al(sizeof(CoopAcc) * 2 * kmax), o_arr = o_bar + al(sizeof(unsigned) * kmax * G * 32),
               bytes = o_arr + al(sizeof(unsigned) * kmax * 32);
  if (!ctx->d_coop_flags) {   // the timeout word (shared with ksg_topo_coop)
    if ((rc = dalloc(ctx, &ctx->d_coop_flags, 8))) return rc;
    ctx->coop_dirty = true;
  }
  if (bytes > ctx->win_bytes) {
    if (ctx->d_win) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)ctx->d_win);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipFree(ctx->d_win);
      ctx->d_win = nullptr;
      ctx->win_bytes = 0;
    }
    if ((rc = dalloc(ctx, &ctx->d_win, bytes))) return rc;
    ctx->win_bytes = bytes;
  }
  char* b = ctx->d_win;
  // flags, partials, atomics sets, counters: zero per run (barrier epochs
  // start from the run's first generation)
  HIPC(ctx, hipMemsetAsync(b, 0, o_tot, ctx->stream));
  HIPC(ctx, hipMemsetAsync(b + o_pod, 0, bytes - o_pod, ctx->stream));
  HIPC(ctx, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(b + o_cur), first, 1, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(b + o_len, wlen.data(), sizeof(int32_t) * count, hipMemcpyHostToDevice, ctx->stream));
  if (ctx->coop_dirty) {   // the timeout word (shared with ksg_topo_coop)
    HIPC(ctx, hipMemsetAsync(ctx->d_coop_flags, 0, 32, ctx->stream));
  }
  CoopArgs a{};
  a.c = ctx->c;
  a.st = ctx->st;
  a.pods = ctx->d_pods;
  a.prog = ctx->d_prog;
  a.profile = d_prof;
  a.G = G;
  a.parts = reinterpret_cast<CoopPart*>(b + o_parts);
  a.phist = reinterpret_cast<int32_t*>(b + o_phist);
  a.acc = reinterpret_cast<CoopAcc*>(b + o_acc);
  a.bar = reinterpret_cast<unsigned*>(b + o_bar);
  a.arrive = reinterpret_cast<unsigned*>(b + o_arr);
  a.pmode = ctx->coop_pmode;
  a.timeout = ctx->d_coop_flags + 4;
  a.commit = 0;
  a.tt = tt;
  a.use_tables = 1;
  a.fused_static = 1;
  a.win_cursor = reinterpret_cast<const int32_t*>(b + o_cur);
  a.win_len = reinterpret_cast<const int32_t*>(b + o_len);
  a.win_base = first;
  a.win_end = first + count;
  a.win_kmax = kmax;
  a.win_tot = reinterpret_cast<int32_t*>(b + o_tot);
  a.win_top = reinterpret_cast<unsigned long long*>(b + o_top);
  a.win_pod = reinterpret_cast<WinPod*>(b + o_pod);
  a.placements = d_pl;
  a.results = d_res;
  a.win_done = reinterpret_cast<unsigned*>(b + o_stats + 64);
  a.win_stats = reinterpret_cast<unsigned long long*>(b + o_stats);
#ifdef KSG_STAMPS
  if (!ctx->d_stamps) {
    if ((rc = dalloc(ctx, &ctx->d_stamps, 16))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_stamps, 0, 128, ctx->stream));
  }
  a.stamps = ctx->d_stamps;
#endif
  *used = true;
  (void)hipGetLastError();
  treset(ctx);
  HIPC(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  if ((rc = tmark(ctx))) return rc;
  unsigned gen = 0;
  int steps = windows_from(0);
  int32_t pos = 0;   // the predicted window's start (the timing's units: node-evals of its rows)
  for (;;) {
    for (int s = 0; s < steps; s++) {
      const int32_t wl = pos < count ? wlen[pos] : 0;
      pos += wl;
      if (++gen >= 0xffffu) {   // barrier epochs are (gen << 16) + k: reset the flags before they wrap
        HIPC(ctx, hipMemsetAsync(b + o_bar, 0, sizeof(unsigned) * kmax * G * 32, ctx->stream));
        gen = 1;
      }
      a.gen = gen;
      if ((ctx->inject_timeout & 1) && pos > 16 && pos - wl < count) {   // test injection: after some windows,
        ctx->inject_timeout &= ~1;                                      // the rows find the timeout word set
        HIPC(ctx, hipMemsetAsync(ctx->d_coop_flags + 4, 0x01, sizeof(unsigned), ctx->stream));
      }
      // rows: the predicted window's length (the rows take min(win_len at the
      // cursor, rows): a window the walk ended early leaves the prediction
      // behind until the host reads the cursor, and a shorter window is valid)
      void* kargs[] = {&a};
      HIPC(ctx, hipLaunchKernel(kf, dim3(G, std::max(wl, 1)), dim3(256), kargs, 0, ctx->stream));
      if ((rc = tlaunched(ctx, KSG_K_TOPO_WIN_ROWS, (double)wl * N))) return rc;
    }
    HIPC(ctx, hipGetLastError());
    int32_t cur = 0;
    unsigned to = 0;
    HIPC(ctx, hipMemcpyAsync(&cur, b + o_cur, sizeof(cur), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(ctx, hipMemcpyAsync(&to, ctx->d_coop_flags + 4, sizeof(to), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(ctx, hipStreamSynchronize(ctx->stream));
    if (to || cur >= first + count) break;   // done, or a row's barrier timed out (run_internal recovers)
    steps = windows_from(cur - first);
    pos = cur - first;
  }
  HIPC(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(ctx->win_stats, b + o_stats, sizeof(ctx->win_stats), hipMemcpyDeviceToHost, ctx->stream));
  return KSG_OK;
}

int flush_stage(ksg_ctx* ctx);
int flush_commit(ksg_ctx* ctx);

// The mutable node state of the context (requested, non-zero requested, pod
// counts, selector counts, domain tables, template totals, host ports) into
// (save) or back from (restore) one device buffer kept across calls: a plain
// topology queue launch whose grid barrier times out has committed some of
// its pods; the call restores the state and relaunches cooperatively.
int state_copy(ksg_ctx* ctx, bool save) {
  const size_t N = ctx->c.N, R = ctx->c.R;
  const struct { void* p; size_t bytes; } part[] = {
      {ctx->st.requested, 8 * R * N},
      {ctx->st.nonzero, 16 * N},
      {ctx->st.pod_count, 4 * N},
      {ctx->st.cnt, 4 * (size_t)std::max(ctx->c.S, 1) * N},
      {ctx->st.tab, 4 * ctx->tab_words},
      {ctx->st.tmpl_total, 4 * (size_t)std::max(ctx->c.n_tmpl, 1)},
      {ctx->st.ports, 4 * (size_t)ctx->c.PW * N},
  };
  size_t total = 0;
  for (const auto& q : part) total += q.p ? (q.bytes + 255) & ~(size_t)255 : 0;
  if (save && total > ctx->state_bak_bytes) {
    if (ctx->d_state_bak) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)ctx->d_state_bak);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipFree(ctx->d_state_bak);
      ctx->d_state_bak = nullptr;
      ctx->state_bak_bytes = 0;
    }
    int rc;
    if ((rc = dalloc(ctx, &ctx->d_state_bak, total))) return rc;
    ctx->state_bak_bytes = total;
  }
  if (!ctx->d_state_bak || total > ctx->state_bak_bytes)
    return fail(ctx, KSG_E_STATE, "state restore without a saved state");
  size_t off = 0;
  for (const auto& q : part) {
    if (!q.p) continue;
    char* b = ctx->d_state_bak + off;
    HIPC(ctx, hipMemcpyAsync(save ? (void*)b : q.p, save ? q.p : (const void*)b, q.bytes, hipMemcpyDeviceToDevice,
                             ctx->stream));
    off += (q.bytes + 255) & ~(size_t)255;
  }
  return KSG_OK;
}

// The capture instances of ksg_topo_coop cover up to 4 nodes per lane
// (coop_kernel): 262,144 nodes on 256 workgroups.
bool coop_capture_fits(const ksg_ctx* ctx) { return ctx->c.N <= 4 * 256 * 256; }

// The device serialiser over a captured chunk (ksched_json.h): lengths,
// offsets, the values; then one copy into the pinned buffer.
int json_serialise(ksg_ctx* ctx, const CapArgs& ca, const ksg_result* d_res, int32_t first, int32_t count) {
  const int N = ctx->c.N;
  if (ctx->json_N != N) return fail(ctx, KSG_E_STATE, "ksg_run_queue_json: no annotator attached for these nodes");
  JsonArgs ja{};
  ja.t = ctx->json_t;
  ja.N = N;
  ja.T = ctx->c.T;
  ja.taints = ctx->c.taints;
  ja.pods = ctx->d_pods;
  ja.first = first;
  ja.res = d_res;
  ja.fstatus = ca.fstatus;
  ja.raw = ca.raw;
  ja.norm = ca.norm;
  ja.n_rows = ca.n_rows;
  for (int p = 0; p < KSG_NPLUGINS; p++) ja.row_of[p] = -1;
  for (int q = 0; q < ca.n_rows; q++) ja.row_of[ca.rows[q]] = q;
  ja.n_filter = ctx->prof.n_filter;
  for (int i = 0; i < KSG_NPLUGINS; i++) ja.filter_order[i] = ctx->prof.filter_order[i];
  ja.score_mask = ctx->prof.score_mask;
  ja.normalize_mask = ctx->json_norm;
  for (int p = 0; p < KSG_NPLUGINS; p++) ja.weight[p] = ctx->json_w[p];
  // segments per pod: enough workgroups for the chip at small chunks
  const int S = std::max(1, std::min(16, (1024 + count - 1) / count));
  ja.count = count;
  ja.S = S;
  const size_t KS = (size_t)count * S;
  // scratch kept across calls (grown only): segment totals and prefixes,
  // value totals, offsets
  const size_t need = 8 * (5 * KS + 6 * KS + 3 * (size_t)count + 3 * (size_t)count + 1) + 8;
  if (need > ctx->json_scratch_bytes) {
    const size_t c = std::max(need, 2 * ctx->json_scratch_bytes);
    if (ctx->d_json_scratch) (void)hipFree(ctx->d_json_scratch);
    ctx->d_json_scratch = nullptr;
    ctx->json_scratch_bytes = 0;
    HIPC(ctx, hipMalloc((void**)&ctx->d_json_scratch, c));
    ctx->json_scratch_bytes = c;
  }
  ja.segtot = reinterpret_cast<int64_t*>(ctx->d_json_scratch);
  ja.segoff = ja.segtot + 5 * KS;
  ja.totals = ja.segoff + 6 * KS;
  ja.offsets = ja.totals + 3 * (size_t)count;
  ja.err = reinterpret_cast<uint32_t*>(ja.offsets + 3 * (size_t)count + 1);
  if (!ctx->json_stream) {
    HIPC(ctx, hipStreamCreateWithFlags(&ctx->json_stream, hipStreamNonBlocking));
    HIPC(ctx, hipEventCreateWithFlags(&ctx->json_written, hipEventDisableTiming));
    for (int q = 0; q < ksg_ctx::kJsonSlots; q++)
      HIPC(ctx, hipEventCreateWithFlags(&ctx->json_copied[q], hipEventDisableTiming));
    HIPC(ctx, hipMalloc((void**)&ctx->d_json_err, sizeof(uint32_t) * ksg_ctx::kJsonSlots));
    HIPC(ctx, hipHostMalloc((void**)&ctx->h_json_err, sizeof(uint32_t) * ksg_ctx::kJsonSlots, hipHostMallocDefault));
  }
  const int slot = ctx->json_next;
  ctx->json_next = (slot + 1) % ksg_ctx::kJsonSlots;
  if (ctx->json_busy[slot]) {   // the copy that last filled this slot (the caller read it two calls ago)
    HIPC(ctx, hipEventSynchronize(ctx->json_copied[slot]));
    ctx->json_busy[slot] = false;
  }
  ja.err = ctx->d_json_err + slot;
  HIPC(ctx, hipMemsetAsync(ja.err, 0, sizeof(uint32_t), ctx->stream));
  hipLaunchKernelGGL(ksg_json_len, dim3(KS), dim3(kJsonBlock), 0, ctx->stream, ja);
  HIPC(ctx, hipGetLastError());
  hipLaunchKernelGGL(ksg_json_scan, dim3(1), dim3(kJsonBlock), 0, ctx->stream, ja);
  HIPC(ctx, hipGetLastError());
  std::vector<int64_t>& joff = ctx->json_off[slot];
  joff.assign(3 * (size_t)count + 1, 0);
  uint32_t err = 0;
  HIPC(ctx, hipMemcpyAsync(joff.data(), ja.offsets, sizeof(int64_t) * joff.size(), hipMemcpyDeviceToHost,
                           ctx->stream));
  HIPC(ctx, hipMemcpyAsync(&err, ja.err, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  if (err) return fail(ctx, KSG_E_INVALID, "ksg_run_queue_json: a status word without a message (or a plugin that did not run)");
  const size_t total = (size_t)joff.back();
  if (total + 1 > ctx->json_out_cap[slot]) {
    const size_t c = std::max(total + 1 + total / 2, ctx->json_out_cap[slot] * 2);
    if (ctx->d_json_out[slot]) (void)hipFree(ctx->d_json_out[slot]);
    ctx->d_json_out[slot] = nullptr;
    ctx->json_out_cap[slot] = 0;
    HIPC(ctx, hipMalloc((void**)&ctx->d_json_out[slot], c));
    ctx->json_out_cap[slot] = c;
  }
  if (total + 1 > ctx->h_json_cap[slot]) {   // grown by half again: pinning is slow, chunks vary a little
    const size_t c = std::max({total + 1 + total / 2, ctx->h_json_cap[slot] + ctx->h_json_cap[slot] / 2,
                               (size_t)1 << 20});
    if (ctx->h_json[slot]) (void)hipHostFree(ctx->h_json[slot]);
    ctx->h_json[slot] = nullptr;
    ctx->h_json_cap[slot] = 0;
    HIPC(ctx, hipHostMalloc((void**)&ctx->h_json[slot], c, hipHostMallocDefault));
    ctx->h_json_cap[slot] = c;
  }
  ja.out = ctx->d_json_out[slot];
  hipLaunchKernelGGL(ksg_json_write, dim3(KS), dim3(kJsonWBlock), 0, ctx->stream, ja);
  HIPC(ctx, hipGetLastError());
  // the copy back on its own stream: the next chunk's kernels overlap it
  HIPC(ctx, hipEventRecord(ctx->json_written, ctx->stream));
  HIPC(ctx, hipStreamWaitEvent(ctx->json_stream, ctx->json_written, 0));
  HIPC(ctx, hipMemcpyAsync(ctx->h_json[slot], ctx->d_json_out[slot], total, hipMemcpyDeviceToHost, ctx->json_stream));
  HIPC(ctx, hipMemcpyAsync(ctx->h_json_err + slot, ja.err, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->json_stream));
  HIPC(ctx, hipEventRecord(ctx->json_copied[slot], ctx->json_stream));
  ctx->json_busy[slot] = true;
  ctx->json_last = slot;
  return KSG_OK;
}

int run_internal(ksg_ctx* ctx, int32_t first, int32_t count, int do_commit, int32_t* placements,
                 ksg_result* results, ksg_capture* cap) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if ((rc = srv_stop(ctx))) return rc;
  if (first < 0 || count < 0 || first + count > ctx->n_pods) return fail(ctx, KSG_E_INVALID, "pod range");
  if ((rc = check_blobs(ctx, first, count))) return rc;
  if ((rc = check_supported(ctx, ctx->prof, first, count))) return rc;
  if (count == 0) return KSG_OK;
  HIPC(ctx, hipSetDevice(ctx->device));
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;
  if (do_commit) ctx->pct_valid = false;   // the queue's assumes bypass the per-cycle tables
  ctx->last_window = false;
  const size_t N = ctx->c.N;
  Tmp tmp;
  ksg_profile* d_prof = nullptr;
  int32_t* d_pl = nullptr;
  ksg_result* d_res = nullptr;
  const bool want_json = ctx->json_want;   // ksg_run_queue_json: the capture stays on the device
  // The serialiser's chunks carve everything from one arena kept across calls:
  // a hipFree waits for the whole device, the previous chunk's copy back included.
  int n_rows = 0;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++) n_rows += (ctx->prof.score_mask >> pl) & 1u;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t arena_parts[8] = {al(sizeof(ksg_profile)), al(sizeof(int32_t) * count), al(sizeof(ksg_result) * count),
                                 al(sizeof(int32_t) * 4 * KSG_BATCH_MAX), al(sizeof(uint32_t) * N * count),
                                 al(sizeof(int64_t) * N * count), al(sizeof(int64_t) * N * n_rows * count),
                                 al(sizeof(int64_t) * N * n_rows * count)};
  char* arena[8] = {};
  if (want_json) {
    size_t need = 0;
    for (size_t b : arena_parts) need += b;
    if (need > ctx->json_arena_bytes) {
      if (ctx->d_json_arena) (void)hipFree(ctx->d_json_arena);
      ctx->d_json_arena = nullptr;
      ctx->json_arena_bytes = 0;
      HIPC(ctx, hipMalloc((void**)&ctx->d_json_arena, need + need / 2));
      ctx->json_arena_bytes = need + need / 2;
    }
    char* b = ctx->d_json_arena;
    for (int i = 0; i < 8; i++) {
      arena[i] = b;
      b += arena_parts[i];
    }
    d_prof = reinterpret_cast<ksg_profile*>(arena[0]);
    d_pl = reinterpret_cast<int32_t*>(arena[1]);
    d_res = reinterpret_cast<ksg_result*>(arena[2]);
  } else {
    TA(tmp, &d_prof, sizeof(ksg_profile));
    TA(tmp, &d_pl, sizeof(int32_t) * count);
    if (results) TA(tmp, &d_res, sizeof(ksg_result) * count);
  }
  HIPC(ctx, hipMemcpyAsync(d_prof, &ctx->prof, sizeof(ksg_profile), hipMemcpyHostToDevice, ctx->stream));
  const bool want_cap = want_json || (cap && (cap->fstatus || cap->raw || cap->norm || cap->total));
  QueueArgs a = base_args(ctx);
  bool batched = do_commit && batch_eligible(ctx, first, count);
  if (ctx->force_path == 1) batched = false;
  // topology pods: the chip-wide path (ksched_topo_coop.h) for placements,
  // ksg_eval (no assume) and captured queues alike
  const bool topo = !batched && needs_topo(ctx, ctx->prof, first, count);
  const bool coop = topo && ctx->topo_coop && ctx->force_path != 1 && !range_has_ports(ctx, first, count) &&
                    (!want_cap || coop_capture_fits(ctx));
  if (want_json && !(batched || coop))
    return fail(ctx, KSG_E_UNSUPPORTED, "ksg_run_queue_json: these pods take neither the batched nor the "
                                        "chip-wide capture path (use ksg_annotate)");
  // captured queues take the batched path too (ksched_capture.h): the capture
  // kernels write the profile's score rows only, in a compact layout (the
  // chip-wide topology path writes the same layout)
  CapArgs ca{};
  if (want_cap && (batched || coop)) {
    ca.c = ctx->c;
    ca.st = ctx->st;
    ca.pods = ctx->d_pods;
    ca.prog = ctx->d_prog;
    ca.prof = d_prof;
    ca.placements = d_pl;
    for (int pl = 0; pl < KSG_NPLUGINS; pl++)
      if ((ctx->prof.score_mask >> pl) & 1u) ca.rows[ca.n_rows++] = pl;
    if (want_json) {
      ca.stats = reinterpret_cast<int32_t*>(arena[3]);
      ca.fstatus = reinterpret_cast<uint32_t*>(arena[4]);
      ca.total = reinterpret_cast<int64_t*>(arena[5]);
      ca.raw = ca.n_rows ? reinterpret_cast<int64_t*>(arena[6]) : nullptr;
      ca.norm = ca.n_rows ? reinterpret_cast<int64_t*>(arena[7]) : nullptr;
    } else {
      TA(tmp, &ca.stats, sizeof(int32_t) * 4 * KSG_BATCH_MAX);
      TA(tmp, &ca.fstatus, sizeof(uint32_t) * N * count);
      TA(tmp, &ca.total, sizeof(int64_t) * N * count);
      if (ca.n_rows) {
        TA(tmp, &ca.raw, sizeof(int64_t) * N * ca.n_rows * count);
        TA(tmp, &ca.norm, sizeof(int64_t) * N * ca.n_rows * count);
      }
    }
  } else if (want_cap) {
    TA(tmp, &a.cap_fstatus, sizeof(uint32_t) * N * count);
    TA(tmp, &a.cap_raw, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    TA(tmp, &a.cap_norm, sizeof(int64_t) * N * KSG_NPLUGINS * count);
    TA(tmp, &a.cap_total, sizeof(int64_t) * N * count);
    HIPC(ctx, hipMemsetAsync(a.cap_raw, 0, sizeof(int64_t) * N * KSG_NPLUGINS * count, ctx->stream));
    HIPC(ctx, hipMemsetAsync(a.cap_norm, 0, sizeof(int64_t) * N * KSG_NPLUGINS * count, ctx->stream));
    HIPC(ctx, hipMemsetAsync(a.cap_total, 0, sizeof(int64_t) * N * count, ctx->stream));
  }
  if (batched) {
    ctx->last_path = 2;
    if ((ctx->batch_mode == 4 || (ctx->batch_mode == 6 && ctx->pipe_window)) && !want_cap) {
      if ((rc = run_pipe(ctx, first, count, d_pl, d_res, d_prof))) return rc;
    } else if ((rc = run_batched(ctx, first, count, d_pl, d_res, want_cap ? &ca : nullptr, d_prof))) {
      return rc;
    }
  } else {
    ctx->last_path = 1;
    a.first = first;
    a.count = count;
    a.do_commit = do_commit;
    a.profiles = d_prof;
    a.placements = d_pl;
    a.results = d_res;
    const int block = N >= 512 ? 512 : 256;   // 512 lanes: <= 256 VGPRs per lane, no spills
    if (coop) {
      ctx->last_path = 4;
      CoopCap cc;
      if (want_cap) {
        cc.mode = 1;
        cc.fs = ca.fstatus;
        cc.raw = reinterpret_cast<char*>(ca.raw);
        cc.norm = reinterpret_cast<char*>(ca.norm);
        cc.tot = reinterpret_cast<char*>(ca.total);
        for (int q = 0; q < ca.n_rows; q++) cc.rows[q] = ca.rows[q];
        cc.n_rows = cc.n_normrows = ca.n_rows;
      }
      // a plain launch relies on the occupancy API for the grid barrier's
      // residency: keep the pre-call node state so that a timeout (the
      // workgroups were not all resident) restores it and relaunches
      // cooperatively instead of failing over partial commits
      if (do_commit && !ctx->coop_launch && (rc = state_copy(ctx, true))) return rc;
      bool win = false;
      if (do_commit && !want_cap && (rc = run_topo_window(ctx, first, count, d_pl, d_res, d_prof, &win))) return rc;
      ctx->last_window = win;
      if (!win && (rc = run_topo_coop(ctx, first, count, d_pl, d_res, d_prof, do_commit, want_cap ? &cc : nullptr)))
        return rc;
    } else if ((rc = launch_queue(ctx, a, 1, block, topo))) {
      return rc;
    }
  }
  if (want_json && (rc = json_serialise(ctx, ca, d_res, first, count))) return rc;
  if (placements) HIPC(ctx, hipMemcpyAsync(placements, d_pl, sizeof(int32_t) * count, hipMemcpyDeviceToHost, ctx->stream));
  if (results) HIPC(ctx, hipMemcpyAsync(results, d_res, sizeof(ksg_result) * count, hipMemcpyDeviceToHost, ctx->stream));
  if (want_json) {
    // nothing else to copy: the values went to the pinned buffer
  } else if (want_cap && (batched || coop)) {
    if (cap->fstatus) HIPC(ctx, hipMemcpyAsync(cap->fstatus, ca.fstatus, sizeof(uint32_t) * N * count, hipMemcpyDeviceToHost, ctx->stream));
    if (cap->total) HIPC(ctx, hipMemcpyAsync(cap->total, ca.total, sizeof(int64_t) * N * count, hipMemcpyDeviceToHost, ctx->stream));
    for (int q = 0; q < ca.n_rows; q++) {   // compact row q -> the caller's plugin row, every pod
      const size_t w = sizeof(int64_t) * N, hp = w * KSG_NPLUGINS, dp = w * ca.n_rows;
      if (cap->raw)
        HIPC(ctx, hipMemcpy2DAsync(cap->raw + (size_t)ca.rows[q] * N, hp, ca.raw + (size_t)q * N, dp, w, count,
                                   hipMemcpyDeviceToHost, ctx->stream));
      if (cap->norm)
        HIPC(ctx, hipMemcpy2DAsync(cap->norm + (size_t)ca.rows[q] * N, hp, ca.norm + (size_t)q * N, dp, w, count,
                                   hipMemcpyDeviceToHost, ctx->stream));
    }
  } else if (want_cap) {
    if (cap->fstatus) HIPC(ctx, hipMemcpyAsync(cap->fstatus, a.cap_fstatus, sizeof(uint32_t) * N * count, hipMemcpyDeviceToHost, ctx->stream));
    if (cap->raw) HIPC(ctx, hipMemcpyAsync(cap->raw, a.cap_raw, sizeof(int64_t) * N * KSG_NPLUGINS * count, hipMemcpyDeviceToHost, ctx->stream));
    if (cap->norm) HIPC(ctx, hipMemcpyAsync(cap->norm, a.cap_norm, sizeof(int64_t) * N * KSG_NPLUGINS * count, hipMemcpyDeviceToHost, ctx->stream));
    if (cap->total) HIPC(ctx, hipMemcpyAsync(cap->total, a.cap_total, sizeof(int64_t) * N * count, hipMemcpyDeviceToHost, ctx->stream));
  }
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIPC(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->last_ms = ms;
  if ((rc = tcollect(ctx))) return rc;
  if (ctx->pipe_tk) {   // the window pipeline's top-k hand-off and the walk's invariant word (run_pipe)
    unsigned tkf[4] = {0, 0, 0, 0};
    HIPC(ctx, hipMemcpy(tkf, ctx->pipe_tk, sizeof(tkf), hipMemcpyDeviceToHost));
    ctx->pipe_tk = nullptr;
    if (tkf[2] == 1 && ctx->last_persist) {
      // the persistent walk waited out its poll for a top-k (a launch it
      // depends on queued behind it): the pre-call state back, then the
      // per-batch form, which launches each walk after its top-k
      if (ctx->stream2) HIPC(ctx, hipStreamSynchronize(ctx->stream2));
      if (do_commit && (rc = state_copy(ctx, false))) return rc;
      ctx->last_persist = false;
      ctx->spec_persist = false;
      ctx->recoveries++;
      return run_internal(ctx, first, count, do_commit, placements, results, cap);
    }
    if (tkf[2] == 1) return fail(ctx, KSG_E_DEVICE, "batched path: top-k hand-off poll timed out");
    if (tkf[2] || tkf[3])
      return fail(ctx, KSG_E_DEVICE, "batched path: speculate-and-verify walk invariant broken (code " +
                                         std::to_string(tkf[3] ? tkf[3] : tkf[2]) + ")");
  }
  if (ctx->last_path == 4) {
    unsigned flags[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPC(ctx, hipMemcpy(flags, ctx->d_coop_flags, sizeof(flags), hipMemcpyDeviceToHost));
    if (flags[4]) {
      ctx->coop_dirty = true;
      if (ctx->coop_launch) return fail(ctx, KSG_E_DEVICE, "topology path: grid barrier timed out (cooperative launch)");
      // not every workgroup was resident: the pre-call state back, then the
      // same call once more with cooperative launches (from now on)
      ctx->coop_launch = true;
      if (do_commit && (rc = state_copy(ctx, false))) return rc;
      ctx->recoveries++;
      return run_internal(ctx, first, count, do_commit, placements, results, cap);
    }
  }
  return KSG_OK;
}

// ---- the per-cycle path ---------------------------------------------------------
// ksg_eval of one pod whose plugins are all node-local (the batched path's
// eligibility): the framework's PreFilter .. NormalizeScore for one pod, as the
// Go shim calls it once per scheduling cycle.  No allocation per call, one
// cooperative launch (ksg_eval_cycle, ksched_cycle.h: N / BLOCK co-resident
// workgroups, one exchange of the pod-wide maxima, every workgroup normalises
// its own nodes, the last to arrive folds the selectHost keys), results
// written by the kernel into a pinned, fine-grained host block, completion
// read from a flag in that block (no copy, no event, no stream
// synchronisation); the host then decodes the result.
// The largest raw NodeAffinity score a pod can get: its preferred terms'
// summed |weight| (program: nterms, then per term weight, nr, nr x {col, op,
// nv, values[nv]}).
int64_t na_pref_bound(const ksg_ctx* ctx, const ksg_pod& p) {
  if (p.na_pref < 0) return 0;
  const int32_t* w = ctx->h_prog.data() + p.na_pref;
  const int32_t* end = ctx->h_prog.data() + p.blob + p.blob_len;
  int64_t s = 0;
  const int nt = *w++;
  for (int t = 0; t < nt && w < end; t++) {
    const int32_t weight = *w++;
    s += weight < 0 ? -(int64_t)weight : weight;
    const int nr = *w++;
    for (int r = 0; r < nr && w + 2 < end; r++) w += 3 + w[2];
  }
  return w <= end ? s : INT64_MAX / 2;   // a malformed program: the widest rows
}

bool eval_fast_eligible(ksg_ctx* ctx, int32_t pod) {
  return ctx->eval_fast && ctx->force_path != 1 && batch_eligible(ctx, pod, 1);
}

int eval_fast(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap, ksg_eval_rows* view = nullptr) {
  std::unique_lock<std::recursive_mutex> srv_lk(g_srv_mu, std::defer_lock);
  if (ctx->srv_mode) srv_lk.lock();   // (g_srv_mu) the whole call: no other context stops this server mid-call
  const size_t N = ctx->c.N;
  const ksg_profile& prof = ctx->prof;
  // score rows: the raw values of every plugin the profile scores.  The
  // normalised TaintToleration / NodeAffinity rows are derived on the host
  // from them and the maxima of the result line, and the totals are not
  // materialised for the view (no reader: the framework sums the weights
  // itself), round 6.
  int rows[KSG_NPLUGINS], n_rows = 0;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    if ((prof.score_mask >> pl) & 1u) rows[n_rows++] = pl;
  // Row width: the narrowest exact one.  Raw Fit / BalancedAllocation /
  // ImageLocality are in [0, 100]; raw TaintToleration is at most the node's
  // taint count, raw NodeAffinity at most the pod's summed preferred weights;
  // none is negative, so one unsigned byte holds them up to 255 (the rows are
  // most of the bytes a cycle writes across the host link).
  const ksg_pod& hp = ctx->h_pods[pod];
  int64_t bound = std::max<int64_t>({(int64_t)100, (int64_t)ctx->c.T, na_pref_bound(ctx, hp)});
  size_t es = bound <= 255 ? 1 : bound < (1 << 15) ? 2 : bound < (1ll << 31) ? 4 : 8;
  int rc;
  HIPC(ctx, hipSetDevice(ctx->device));
  // one-wave workgroups, KN nodes per lane: the smallest KN whose grid is
  // co-resident (the exchange needs every workgroup resident)
  auto kernel_of = [&](int kn) -> const void* {
    if (ctx->cycle_sys) {
      if (kn == 1) return (const void*)ksg_eval_cycle<1, true>;
      if (kn == 2) return (const void*)ksg_eval_cycle<2, true>;
      return (const void*)ksg_eval_cycle<4, true>;
    }
    if (kn == 1) return (const void*)ksg_eval_cycle<1, false>;
    if (kn == 2) return (const void*)ksg_eval_cycle<2, false>;
    return (const void*)ksg_eval_cycle<4, false>;
  };
  int kn = ctx->cycle_kn;
  for (;; kn *= 2) {
    const int bi = kn == 1 ? 0 : kn == 2 ? 1 : 2;
    if (!ctx->cycle_cap[bi]) {
      int per_cu = 0;
      HIPC(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel_of(kn), 64, 0));
      hipDeviceProp_t dp;
      HIPC(ctx, hipGetDeviceProperties(&dp, ctx->device));
      // one fewer than the API's answer per CU (MI355X guide: the hardware may admit one fewer)
      ctx->cycle_cap[bi] = std::max(1, per_cu - 1) * dp.multiProcessorCount;
    }
    if ((N + 64 * kn - 1) / (64 * kn) <= (size_t)ctx->cycle_cap[bi]) break;
    if (kn == kCycMaxKN) return fail(ctx, KSG_E_UNSUPPORTED, "per-cycle evaluation: grid not co-resident");
  }
  const unsigned G = (unsigned)((N + 64 * kn - 1) / (64 * kn));
  const size_t Gm = (N + 63) / 64;   // the largest grid (KN = 1): no reallocation on a KN change
  // host block: result line (stats[4], best key, error bits, done) | pad | fstatus[N] | raw[n_rows][N]
  const size_t o_fs = 64, o_raw = o_fs + ((4 * N + 7) & ~(size_t)7);
  const size_t h_need = o_raw + es * N * std::max(n_rows, 1);
  // device block: exchange lines [Gm][32] | timeout | completion counter | key slot, error slot
  const size_t d_flags = 0, d_to = d_flags + 128 * Gm, d_arr = d_to + 128, d_key = d_arr + 128;
  const size_t d_need = d_key + 128;
  if (G != ctx->cyc_last_G) ctx->ev_clean = false;   // the counter counts in multiples of G
  ctx->cyc_last_G = G;
  if (d_need > ctx->ev_bytes || h_need > ctx->h_ev_bytes || !ctx->ev_clean || ctx->ev_prof_dirty || !ctx->d_ev_prof)
    if ((rc = srv_stop(ctx))) return rc;   // stream work ahead: a running server leaves first
  if (d_need > ctx->ev_bytes) {
    if (ctx->d_ev) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)ctx->d_ev);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipFree(ctx->d_ev);
      ctx->d_ev = nullptr;
    }
    if ((rc = dalloc(ctx, &ctx->d_ev, d_need))) return rc;
    ctx->ev_bytes = d_need;
    ctx->ev_clean = false;
  }
  if (!ctx->d_ev_prof && (rc = dalloc(ctx, &ctx->d_ev_prof, 1))) return rc;
  if (h_need > ctx->h_ev_bytes) {
    if (ctx->h_ev) {
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipHostFree(ctx->h_ev);
      ctx->h_ev = nullptr;
      ctx->h_ev_bytes = 0;
    }
    HIPC(ctx, hipHostMalloc((void**)&ctx->h_ev, h_need, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(ctx->h_ev, 0, h_need);   // done words: no call's sequence number is 0
    ctx->h_ev_bytes = h_need;
    void* dp = nullptr;
    HIPC(ctx, hipHostGetDevicePointer(&dp, ctx->h_ev, 0));
    ctx->d_hev = static_cast<char*>(dp);
  }
  if (!ctx->ev_clean) {   // exchange flags (no call's sequence number is 0) and the timeout word
    HIPC(ctx, hipMemsetAsync(ctx->d_ev + d_flags, 0, d_need - d_flags, ctx->stream));
    ctx->ev_clean = true;
  }
  if (ctx->ev_prof_dirty) {
    HIPC(ctx, hipMemcpyAsync(ctx->d_ev_prof, &ctx->prof, sizeof(ksg_profile), hipMemcpyHostToDevice, ctx->stream));
    ctx->ev_prof_dirty = false;
  }
  // the pod's append still staged: read from the staging buffer by the
  // kernel (its programs must all lie in the staged words)
  const bool staged = ctx->stage_pending && ctx->stage_n == 1 && ctx->stage_first == pod && ctx->d_stage &&
                      hp.blob >= ctx->stage_base && (int64_t)hp.blob + hp.blob_len <= ctx->stage_base + ctx->stage_len &&
                      (hp.node_set < 0 || (hp.node_set >= ctx->stage_base &&
                                           (int64_t)hp.node_set + ((int64_t)N + 31) / 32 <= ctx->stage_base + ctx->stage_len));
  if (!staged && (rc = flush_stage(ctx))) return rc;
  char* hb = ctx->h_ev;
  char* db = ctx->d_hev;
  // The arguments: the static part (what the persistent server keeps) and this
  // call (the pod, its profile facts, the deferred assume, the outputs)
  CycArgs& ca = ctx->cyc_args;
  CycStatic& cs = ca.s;
  cs.c = ctx->c;
  cs.requested = ctx->st.requested;
  cs.nonzero = ctx->st.nonzero;
  cs.pod_count = ctx->st.pod_count;
  cs.used_ports = ctx->st.ports;
  cs.flags = reinterpret_cast<unsigned*>(ctx->d_ev + d_flags);
  cs.timeout = reinterpret_cast<unsigned*>(ctx->d_ev + d_to);
  cs.arrive = reinterpret_cast<unsigned*>(ctx->d_ev + d_arr);
  cs.key = reinterpret_cast<unsigned long long*>(ctx->d_ev + d_key);
  cs.errw = reinterpret_cast<unsigned*>(ctx->d_ev + d_key + 16);
  cs.stamps = nullptr;
#ifdef KSG_STAMPS
  if (!ctx->d_stamps) {
    if ((rc = srv_stop(ctx))) return rc;
    if ((rc = dalloc(ctx, &ctx->d_stamps, 16))) return rc;
    HIPC(ctx, hipMemsetAsync(ctx->d_stamps, 0, 128, ctx->stream));
  }
  cs.stamps = ctx->d_stamps;
#endif
  const bool want_img = ((prof.score_mask >> KSG_PL_IMAGE_LOCALITY) & 1u) && ctx->c.I > 0;
  const bool server = ctx->srv_mode;
  if (ctx->srv_running) {   // a server launched for other arguments, or idle long enough to be near its own exit
    const double idle = std::chrono::duration<double>(std::chrono::steady_clock::now() - ctx->srv_last).count();
    if (!server || ctx->srv_kn != kn || ctx->srv_G != G || ctx->srv_img != want_img || ctx->srv_sys != ctx->cycle_sys ||
        idle > 0.05 || std::memcmp(&ctx->srv_static, &cs, sizeof(CycStatic)) != 0)
      if ((rc = srv_stop(ctx))) return rc;
  }
  // test injection: this launch's exchange finds the sticky timeout word set
  // (the one-launch form; a server polls the word while idle and would leave)
  if ((ctx->inject_timeout & 8) && !server && !ctx->cycle_coop) {
    ctx->inject_timeout &= ~8;
    HIPC(ctx, hipMemsetAsync(ctx->d_ev + d_to, 0x01, sizeof(unsigned), ctx->stream));
  }
  if (server && !ctx->srv_running) {   // the persistent form: started once, fed through the mailbox
    if (g_srv_ctx && g_srv_ctx != ctx && (rc = srv_stop(g_srv_ctx))) return rc;   // one server per process
    if (!ctx->h_mb) {
      // The mailbox in fine-grained device memory when the CPU can write it
      // (large BAR: the allocation is mapped writable into this process):
      // the workgroups then poll HBM instead of reading host memory across
      // PCIe, and each reads the call itself (no relay through workgroup 0).
      // scripts/probe_mailbox.hip: 2.97 vs 5.86 us per host -> GPU -> host
      // round trip with a 640-byte call.  Else pinned host memory + relay.
      void* dm = nullptr;
      if (!getenv("KSG_SRV_HOST_MAILBOX") &&
          hipExtMallocWithFlags(&dm, sizeof(SrvMailbox), hipDeviceMallocFinegrained) == hipSuccess) {
        hipPointerAttribute_t at{};
        void* hp = hipPointerGetAttributes(&at, dm) == hipSuccess && at.hostPointer ? at.hostPointer : dm;
        if (host_writable(hp, sizeof(SrvMailbox))) {
          ctx->h_mb = static_cast<SrvMailbox*>(hp);
          ctx->d_mb = static_cast<const SrvMailbox*>(dm);
          ctx->mb_device = true;
          ctx->mb_alloc = dm;
        } else {
          (void)hipFree(dm);
        }
      }
      if (!ctx->h_mb) {
        HIPC(ctx, hipHostMalloc((void**)&ctx->h_mb, sizeof(SrvMailbox), hipHostMallocMapped | hipHostMallocCoherent));
        void* dp = nullptr;
        HIPC(ctx, hipHostGetDevicePointer(&dp, ctx->h_mb, 0));
        ctx->d_mb = static_cast<const SrvMailbox*>(dp);
        ctx->mb_device = false;
      }
      std::memset(ctx->h_mb, 0, sizeof(SrvMailbox));
      std::atomic_thread_fence(std::memory_order_seq_cst);
      __builtin_ia32_sfence();
    }
    if (!ctx->d_srv) {   // the relay: call | programs | go word (zeroed: no sequence number is 0)
      if ((rc = dalloc(ctx, &ctx->d_srv, sizeof(CycCall) + sizeof(int32_t) * KSG_BLOB_MAX + 128))) return rc;
      HIPC(ctx, hipMemsetAsync(ctx->d_srv, 0, sizeof(CycCall) + sizeof(int32_t) * KSG_BLOB_MAX + 128, ctx->stream));
    }
    SrvArgs sa{};
    sa.s = cs;
    sa.mb = ctx->d_mb;
    sa.d_call = reinterpret_cast<CycCall*>(ctx->d_srv);
    sa.d_blob = reinterpret_cast<int32_t*>(ctx->d_srv + sizeof(CycCall));
    sa.d_go = reinterpret_cast<unsigned*>(ctx->d_srv + sizeof(CycCall) + sizeof(int32_t) * KSG_BLOB_MAX);
    sa.last = __atomic_load_n(&ctx->h_mb->seq, __ATOMIC_ACQUIRE);
    sa.want_img = want_img;
    sa.direct = ctx->mb_device ? 1 : 0;
    // the relay's go word starts at the last sequence number served: the
    // workgroups other than 0 take any other value for a relayed call (a relay
    // block reallocated and zeroed by a reload, with the mailbox's sequence
    // past 0, read as one: a zeroed call, an illegal address)
    HIPC(ctx, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sa.d_go), (int)sa.last, 1, ctx->stream));
    void* sargs[] = {&sa};
    const void* kf = ctx->cycle_sys ? (kn == 1 ? (const void*)ksg_cycle_server<1, true>
                                      : kn == 2 ? (const void*)ksg_cycle_server<2, true>
                                                : (const void*)ksg_cycle_server<4, true>)
                                    : (kn == 1 ? (const void*)ksg_cycle_server<1, false>
                                      : kn == 2 ? (const void*)ksg_cycle_server<2, false>
                                                : (const void*)ksg_cycle_server<4, false>);
    // plain, G within the occupancy API's residency, as the per-cycle launch
    // (a process that made cooperative launches faults in the runtime's exit
    // teardown under rocprofv3); an exchange timeout ends the server and the
    // next one launches cooperatively (the runtime's residency guarantee)
    if (ctx->cycle_coop)
      HIPC(ctx, hipLaunchCooperativeKernel(kf, dim3(G), dim3(64), sargs, 0, ctx->stream));
    else
      HIPC(ctx, hipLaunchKernel(kf, dim3(G), dim3(64), sargs, 0, ctx->stream));
    HIPC(ctx, hipGetLastError());
    ctx->srv_running = true;
    g_srv_ctx = ctx;
    ctx->srv_last = std::chrono::steady_clock::now();
    ctx->srv_kn = kn;
    ctx->srv_G = G;
    ctx->srv_img = want_img;
    ctx->srv_sys = ctx->cycle_sys;
    ctx->srv_static = cs;
  }
  const unsigned seq = ++ctx->ev_seq == 0 ? ++ctx->ev_seq : ctx->ev_seq;   // never 0 (a fresh block)
  CycCall& ck = ca.k;
  ck.pod = hp;
  // the profile facts of this pod (make_view(topo = false) + cm_prof, on the host)
  {
    uint32_t fskip = hp.filter_skip | (1u << KSG_PL_INTER_POD_AFFINITY) | (1u << KSG_PL_POD_TOPOLOGY_SPREAD);
    ck.forder = 0;
    ck.fmask = 0;
    ck.n_filter = prof.n_filter;
    for (int kf = 0; kf < prof.n_filter; kf++) {
      const int pl = prof.filter_order[kf];
      ck.forder |= (uint64_t)(pl & 15) << (4 * kf);
      if (!((fskip >> pl) & 1u)) ck.fmask |= 1u << pl;
    }
    ck.smask = prof.score_mask & ~hp.score_skip &
               ~((1u << KSG_PL_INTER_POD_AFFINITY) | (1u << KSG_PL_POD_TOPOLOGY_SPREAD));
    ck.w_fit = prof.weight[KSG_PL_NODE_RESOURCES_FIT];
    ck.w_ba = prof.weight[KSG_PL_BALANCED_ALLOCATION];
    ck.w_img = prof.weight[KSG_PL_IMAGE_LOCALITY];
    ck.w_t = prof.weight[KSG_PL_TAINT_TOLERATION];
    ck.w_a = prof.weight[KSG_PL_NODE_AFFINITY];
    ck.fit_ignored = prof.fit_ignored_res;
    bool ok = prof.fit_n == 2 && prof.ba_n == 2;   // cm_prof (ksched_device.h)
    int64_t wc = 0, wm = 0;
    if (ok) {
      const int r0 = prof.fit_res[0], r1 = prof.fit_res[1];
      ok = (r0 == KSG_RES_CPU && r1 == KSG_RES_MEM) || (r0 == KSG_RES_MEM && r1 == KSG_RES_CPU);
      wc = r0 == KSG_RES_CPU ? prof.fit_w[0] : prof.fit_w[1];
      wm = r0 == KSG_RES_CPU ? prof.fit_w[1] : prof.fit_w[0];
      const int b0 = prof.ba_res[0], b1 = prof.ba_res[1];
      ok = ok && ((b0 == KSG_RES_CPU && b1 == KSG_RES_MEM) || (b0 == KSG_RES_MEM && b1 == KSG_RES_CPU));
      ok = ok && wc > 0 && wm > 0 && prof.fit_strategy != KSG_REQUESTED_TO_CAPACITY_RATIO;
    }
    ck.cm_fast = ok;
    ck.cm_least = prof.fit_strategy == KSG_LEAST_ALLOCATED;
    ck.cm_wc = ok ? wc : 0;
    ck.cm_wm = ok ? wm : 0;
    ck.cm_inv_ws = ok ? 1.0f / (float)(wc + wm) : 1.0f;
    ck.cm_inv_wc = ok ? 1.0f / (float)wc : 1.0f;
    ck.cm_inv_wm = ok ? 1.0f / (float)wm : 1.0f;
  }
  ck.gprof = ctx->d_ev_prof;
  ck.n_rows = n_rows;
  ck.es = (int32_t)es;
  ck.kn = kn;
  ck.rows = 0;
  for (int q = 0; q < n_rows; q++) ck.rows |= (uint64_t)(rows[q] & 15) << (4 * q);
  ck.h_fs = reinterpret_cast<uint32_t*>(db + o_fs);
  ck.h_raw = db + o_raw;
  ck.h_stats = reinterpret_cast<int32_t*>(db);
  ck.seq = seq;
  ck.op = 0;
  // the pod's programs: inline (kernel arguments or mailbox, from the host
  // copy) when they fit, else read by the kernel from the staged append or
  // the device pool
  const int32_t* sprog = staged ? reinterpret_cast<const int32_t*>(ctx->d_stage + sizeof(ksg_pod)) : nullptr;
  ck.gprog = staged ? sprog - ctx->stage_base : ctx->d_prog;
  ck.blob_len = hp.blob_len;
  ck.bsrc = ck.gprog + hp.blob;
  if (hp.blob < 0 || (size_t)hp.blob + hp.blob_len > ctx->h_prog.size())
    return fail(ctx, KSG_E_STATE, "per-cycle evaluation: pod programs outside the host program copy");
  ck.wpods = nullptr;
  if (staged) {
    ck.wpods = ctx->d_pods + pod;
    ck.wprog = ctx->d_prog + ctx->stage_base;
    ck.sprog = sprog;
    ck.slen = ctx->stage_len;
  }
  ck.cm_node = -1;
  if (ctx->pc_node >= 0) {   // the deferred assume: the node's owner lane adds it before evaluating
    const ksg_pod& q = ctx->h_pods[ctx->pc_pod];
    ck.cm_node = ctx->pc_node;
    for (int r = 0; r < KSG_MAX_RES; r++) ck.cm_req[r] = q.req[r];
    ck.cm_nz_cpu = q.nz_cpu;
    ck.cm_nz_mem = q.nz_mem;
  }
  if (server) {
    // the call, then its sequence number (x86 stores are ordered; the server
    // reads seq, then the rest)
    SrvMailbox* mb = ctx->h_mb;
    std::memcpy(&mb->k, &ck, sizeof(CycCall));
    std::memcpy(mb->blob, ctx->h_prog.data() + hp.blob, sizeof(int32_t) * hp.blob_len);
    __builtin_ia32_sfence();   // (in case a copy used streaming stores)
    __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
  } else {
    if (hp.blob_len <= kCycBlob) std::memcpy(ca.blob, ctx->h_prog.data() + hp.blob, sizeof(int32_t) * hp.blob_len);
    treset(ctx);
    if ((rc = tmark(ctx))) return rc;
    void* kargs[] = {&ca};
    if (ctx->cycle_coop)
      HIPC(ctx, hipLaunchCooperativeKernel(kernel_of(kn), dim3(G), dim3(64), kargs, 0, ctx->stream));
    else   // G is within the occupancy API's co-resident count less one per CU (the exchange's poll is bounded)
      HIPC(ctx, hipLaunchKernel(kernel_of(kn), dim3(G), dim3(64), kargs, 0, ctx->stream));
    if ((rc = tlaunched(ctx, KSG_K_EVAL_CYCLE, (double)N))) return rc;
    HIPC(ctx, hipGetLastError());
  }
  ctx->pc_node = -1;   // applied by this call (a retry below must not add it again)
  // the staged append is consumed: the kernel read it (or had it with the
  // launch) before its workgroups stored their done words, which this call
  // waits for, so the staging buffer is free when it returns (no event)
  if (staged) ctx->stage_pending = false;
  // the last workgroup stores the result line and then seq into its done word
  // (after every workgroup's rows): spin on it, checking the stream now and
  // then (a failed launch never stores it)
  const volatile int32_t* line = reinterpret_cast<const volatile int32_t*>(hb);
  for (unsigned spins = 0; (unsigned)line[7] != seq; spins++) {
    __builtin_ia32_pause();
    if ((spins & 1023) == 1023) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess && (unsigned)line[7] != seq) {
        ctx->ev_clean = false;
        ctx->srv_running = false;
        return fail(ctx, KSG_E_DEVICE, server ? "per-cycle server: left without serving the call"
                                              : "per-cycle evaluation: kernel finished without its completion word");
      }
      if (e != hipSuccess && e != hipErrorNotReady)
        return fail(ctx, KSG_E_DEVICE, std::string("per-cycle evaluation: ") + hipGetErrorString(e));
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  if ((rc = tcollect(ctx))) return rc;
  const int32_t* st = reinterpret_cast<const int32_t*>(hb);
  const int32_t nfeas = st[0];
  unsigned long long best;
  std::memcpy(&best, st + 4, 8);
  const uint32_t herr = (uint32_t)st[6];
  if (server) ctx->srv_last = std::chrono::steady_clock::now();
  if (herr & 2u) {
    ctx->ev_clean = false;   // clears the sticky timeout word before the next call
    if (server) {            // every workgroup of the server leaves on a timed-out exchange
      (void)hipStreamSynchronize(ctx->stream);
      ctx->srv_running = false;
      if (!ctx->cycle_coop) {   // not every workgroup was resident: a cooperative server from now on
        ctx->cycle_coop = true;
        ctx->recoveries++;
        return eval_fast(ctx, pod, res, cap, view);
      }
      return fail(ctx, KSG_E_DEVICE, "per-cycle server: workgroup exchange timed out");
    }
    if (!ctx->cycle_coop) {   // not every workgroup was resident: the cooperative launch from now on
      ctx->cycle_coop = true;
      ctx->recoveries++;
      return eval_fast(ctx, pod, res, cap, view);
    }
    return fail(ctx, KSG_E_DEVICE, "per-cycle evaluation: workgroup exchange timed out");
  }
  uint32_t status = 0;
  int32_t selected = -1;
  if (nfeas == 1) {
    selected = (int32_t)N - st[3];
  } else if (nfeas >= 2) {
    status |= KSG_ST_SCORED;
    if (herr & 1u) status |= KSG_ST_SCORE_ERROR;
    else selected = (int32_t)(0xffffffffu - (uint32_t)(best & 0xffffffffu));
  }
  // ipa_skip_bits (ksched_kernels.h) on the host: the pod carries no
  // InterPodAffinity program on this path
  uint32_t score_skip = hp.score_skip;
  bool ipa_filter = false;
  for (int kf = 0; kf < prof.n_filter; kf++) ipa_filter |= prof.filter_order[kf] == KSG_PL_INTER_POD_AFFINITY;
  if (hp.ipa < 0) {
    if (ipa_filter) status |= KSG_ST_IPA_PREFILTER_SKIP;
    if ((status & KSG_ST_SCORED) && ((prof.score_mask >> KSG_PL_INTER_POD_AFFINITY) & 1u) &&
        !((hp.score_skip >> KSG_PL_INTER_POD_AFFINITY) & 1u)) {
      status |= KSG_ST_IPA_PRESCORE_SKIP;
      score_skip |= 1u << KSG_PL_INTER_POD_AFFINITY;
    }
  }
  res->selected = selected;
  res->n_feasible = nfeas;
  res->status = status;
  res->score_skip = score_skip;
  auto row_at = [&](int q, size_t n) -> int64_t {   // raw row q at node n
    const char* r = hb + o_raw + es * N * q;
    return es == 1   ? reinterpret_cast<const uint8_t*>(r)[n]
           : es == 2 ? reinterpret_cast<const int16_t*>(r)[n]
           : es == 4 ? reinterpret_cast<const int32_t*>(r)[n] : reinterpret_cast<const int64_t*>(r)[n];
  };
  // DefaultNormalizeScore of TaintToleration (reverse) / NodeAffinity from
  // the raw value and the device's maximum over the feasible nodes (the
  // kernel's total_score arithmetic); 0 where nothing was scored
  const int64_t max_t = st[1], max_a = st[2];
  const uint32_t smask = prof.score_mask & ~hp.score_skip;
  auto norm_of = [&](int pl, int64_t raw) -> int64_t {
    if (!((smask >> pl) & 1u)) return 0;
    if (pl == KSG_PL_TAINT_TOLERATION) return max_t != 0 ? 100 - (100 * raw) / max_t : 100;
    if (pl == KSG_PL_NODE_AFFINITY) return max_a != 0 ? (100 * raw) / max_a : raw;
    return raw;
  };
  const bool scored = (status & KSG_ST_SCORED) != 0;
  if (view) {   // the rows where the kernel wrote them
    *view = ksg_eval_rows{};
    view->n_nodes = (int32_t)N;
    view->elem_bytes = (int32_t)es;
    view->fstatus = reinterpret_cast<const uint32_t*>(hb + o_fs);
    for (int q = 0; q < n_rows; q++) {
      const int pl = rows[q];
      view->raw[pl] = hb + o_raw + es * N * q;
      const bool derived = pl == KSG_PL_TAINT_TOLERATION || pl == KSG_PL_NODE_AFFINITY;
      view->norm[pl] = derived ? nullptr : view->raw[pl];
      if (derived) {
        view->norm_from_raw |= 1u << pl;
        view->norm_max[pl] = pl == KSG_PL_TAINT_TOLERATION ? max_t : max_a;
      }
    }
    view->norm_scored = scored ? smask : 0u;
    view->total = nullptr;
  }
  const bool want_raw = cap && cap->raw, want_norm = cap && cap->norm, want_tot = cap && cap->total;
  if (cap && cap->fstatus) std::memcpy(cap->fstatus, hb + o_fs, 4 * N);
  if (want_tot) std::memset(cap->total, 0, 8 * N);
  const uint32_t* fs = reinterpret_cast<const uint32_t*>(hb + o_fs);
  for (int q = 0; q < n_rows && (want_raw || want_norm || want_tot); q++) {   // (a view alone: nothing to copy)
    const int pl = rows[q];
    int64_t* dr = want_raw ? cap->raw + (size_t)pl * N : nullptr;
    int64_t* dn = want_norm ? cap->norm + (size_t)pl * N : nullptr;
    const int64_t w = prof.weight[pl];
    for (size_t n = 0; n < N; n++) {
      const int64_t raw = row_at(q, n);
      if (dr) dr[n] = raw;
      // plugins without ScoreExtensions record the raw score as the final one
      const int64_t v = scored && fs[n] == 0 ? norm_of(pl, raw) : 0;
      if (dn) dn[n] = v;
      if (want_tot) cap->total[n] += v * w;
    }
  }
  ctx->last_path = 5;
  return KSG_OK;
}

// ---- the per-cycle path of a topology pod ------------------------------------------
// ksg_eval of one PodTopologySpread / InterPodAffinity pod: the chip-wide
// topology kernel (ksched_topo_coop.h, its per-cycle capture instance CAP = 2)
// evaluates the pod without assuming it and writes the status words, the
// profile's score rows (int64) and the result into the pinned host block the
// caller reads in place, then sets the flag; no copy, no event.
bool eval_topo_eligible(ksg_ctx* ctx, int32_t pod) {
  return ctx->eval_fast && ctx->topo_coop && ctx->force_path != 1 && needs_topo(ctx, ctx->prof, pod, 1) &&
         !range_has_ports(ctx, pod, 1) && coop_capture_fits(ctx) && check_supported(ctx, ctx->prof, pod, 1) == KSG_OK;
}

int eval_topo_fast(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap, ksg_eval_rows* view = nullptr,
                   int es = 2) {
  const size_t N = ctx->c.N;
  const ksg_profile& prof = ctx->prof;
  int rows[KSG_NPLUGINS], n_rows = 0, n_normrows = 0;
  for (int pl : {KSG_PL_TAINT_TOLERATION, KSG_PL_NODE_AFFINITY, KSG_PL_POD_TOPOLOGY_SPREAD, KSG_PL_INTER_POD_AFFINITY})
    if ((prof.score_mask >> pl) & 1u) rows[n_rows++] = pl;
  n_normrows = n_rows;
  for (int pl = 0; pl < KSG_NPLUGINS; pl++)
    if (((prof.score_mask >> pl) & 1u) && pl != KSG_PL_TAINT_TOLERATION && pl != KSG_PL_NODE_AFFINITY &&
        pl != KSG_PL_POD_TOPOLOGY_SPREAD && pl != KSG_PL_INTER_POD_AFFINITY)
      rows[n_rows++] = pl;
  // Row width es: 2 bytes first (every score of the default weights fits);
  // the kernel flags a value that does not fit (raw PodTopologySpread /
  // InterPodAffinity scores have no fixed range) and the pod is evaluated
  // again at 4, then 8 bytes.  The block is sized for 8.
  // host block: result (16 B) .. overflow word at 24, flag at 28 | fstatus[N] | raw[n_rows][N] | total[N] |
  // norm[n_normrows][N]
  const size_t o_fs = 32, o_raw = o_fs + ((4 * N + 7) & ~(size_t)7);
  const size_t o_tot = o_raw + ((es * N * n_rows + 7) & ~(size_t)7), o_norm = o_tot + ((es * N + 7) & ~(size_t)7);
  const size_t h_need = o_raw + 8 * N * (n_rows + 1 + std::max(n_normrows, 1)) + 64;
  int rc;
  HIPC(ctx, hipSetDevice(ctx->device));
  // the pod's append still staged: the kernel reads it from the staging
  // buffer and copies it to the device pool (no copy launches in front of it)
  const ksg_pod& hp = ctx->h_pods[pod];
  const bool staged = ctx->stage_pending && ctx->stage_n == 1 && ctx->stage_first == pod && ctx->d_stage &&
                      hp.blob >= ctx->stage_base && (int64_t)hp.blob + hp.blob_len <= ctx->stage_base + ctx->stage_len &&
                      (hp.node_set < 0 || (hp.node_set >= ctx->stage_base &&
                                           (int64_t)hp.node_set + ((int64_t)N + 31) / 32 <= ctx->stage_base + ctx->stage_len));
  if (!staged && (rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;
  if (!ctx->d_ev_prof && (rc = dalloc(ctx, &ctx->d_ev_prof, 1))) return rc;
  if (!ctx->d_ev_pl && (rc = dalloc(ctx, &ctx->d_ev_pl, 4))) return rc;
  if (h_need > ctx->h_evt_bytes) {
    if (ctx->h_evt) {
      HIPC(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipHostFree(ctx->h_evt);
      ctx->h_evt = nullptr;
      ctx->h_evt_bytes = 0;
    }
    HIPC(ctx, hipHostMalloc((void**)&ctx->h_evt, h_need, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(ctx->h_evt, 0, h_need);
    ctx->h_evt_bytes = h_need;
    void* dp = nullptr;
    HIPC(ctx, hipHostGetDevicePointer(&dp, ctx->h_evt, 0));
    ctx->d_hevt = static_cast<char*>(dp);
  }
  if (ctx->ev_prof_dirty) {
    HIPC(ctx, hipMemcpyAsync(ctx->d_ev_prof, &ctx->prof, sizeof(ksg_profile), hipMemcpyHostToDevice, ctx->stream));
    ctx->ev_prof_dirty = false;
  }
  char* hb = ctx->h_evt;
  char* db = ctx->d_hevt;
  volatile unsigned* flag = reinterpret_cast<volatile unsigned*>(hb + 28);
  const unsigned seq = ++ctx->ev_seq == 0 ? ++ctx->ev_seq : ctx->ev_seq;
  CoopCap cc;
  cc.mode = 2;
  cc.fs = reinterpret_cast<uint32_t*>(db + o_fs);
  cc.raw = db + o_raw;
  cc.norm = db + o_norm;
  cc.tot = db + o_tot;
  for (int q = 0; q < n_rows; q++) cc.rows[q] = rows[q];
  cc.n_rows = n_rows;
  cc.n_normrows = n_normrows;
  cc.narrow = 0;
  cc.es = es;
  cc.h_res = reinterpret_cast<ksg_result*>(db);
  cc.h_ovf = reinterpret_cast<unsigned*>(db + 24);
  cc.h_flag = reinterpret_cast<unsigned*>(db + 28);
  cc.seq = seq;
  if (staged) {
    cc.stage = ctx->d_stage;
    cc.stage_base = ctx->stage_base;
    cc.stage_len = ctx->stage_len;
  }
  if ((rc = run_topo_coop(ctx, pod, 1, ctx->d_ev_pl, nullptr, ctx->d_ev_prof, 0, &cc, false))) {
    ctx->coop_dirty = true;
    return rc;
  }
  if (staged) ctx->stage_pending = false;   // the kernel's workgroup 0 writes it to the device pool
  for (unsigned spins = 0; *flag != seq; spins++) {
    __builtin_ia32_pause();
    if ((spins & 1023) == 1023) {
      const hipError_t e = hipStreamQuery(ctx->stream);
      if (e == hipSuccess && *flag != seq) {
        ctx->coop_dirty = true;   // a grid barrier timed out: the flags and atomics sets are reset next time
        if (!ctx->topo_eval_coop) {   // not every workgroup was resident: cooperative launches from now on
          ctx->topo_eval_coop = true;
          ctx->recoveries++;
          return eval_topo_fast(ctx, pod, res, cap, view, es);
        }
        return fail(ctx, KSG_E_DEVICE, "per-cycle topology evaluation: kernel finished without its completion flag "
                                       "(grid barrier timed out)");
      }
      if (e != hipSuccess && e != hipErrorNotReady) {
        ctx->coop_dirty = true;
        return fail(ctx, KSG_E_DEVICE, std::string("per-cycle topology evaluation: ") + hipGetErrorString(e));
      }
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  if ((rc = tcollect(ctx))) return rc;
  if (*reinterpret_cast<const volatile unsigned*>(hb + 24) && es < 8)   // a value wider than the rows
    return eval_topo_fast(ctx, pod, res, cap, view, es * 2);
  *res = *reinterpret_cast<const ksg_result*>(hb);
  auto put_row = [&](int64_t* dst, size_t off) {   // one row into the caller's int64 array
    if (es == 2) {
      const int16_t* src = reinterpret_cast<const int16_t*>(hb + off);
      for (size_t n = 0; n < N; n++) dst[n] = src[n];
    } else if (es == 4) {
      const int32_t* src = reinterpret_cast<const int32_t*>(hb + off);
      for (size_t n = 0; n < N; n++) dst[n] = src[n];
    } else {
      std::memcpy(dst, hb + off, 8 * N);
    }
  };
  if (view) {
    *view = ksg_eval_rows{};
    view->n_nodes = (int32_t)N;
    view->elem_bytes = (int32_t)es;
    view->fstatus = reinterpret_cast<const uint32_t*>(hb + o_fs);
    for (int q = 0; q < n_rows; q++) {
      view->raw[rows[q]] = hb + o_raw + es * N * q;
      view->norm[rows[q]] = q < n_normrows ? hb + o_norm + es * N * q : view->raw[rows[q]];
    }
    view->total = hb + o_tot;
  }
  if (cap) {
    if (cap->fstatus) std::memcpy(cap->fstatus, hb + o_fs, 4 * N);
    for (int q = 0; q < n_rows; q++) {
      if (cap->raw) put_row(cap->raw + (size_t)rows[q] * N, o_raw + es * N * q);
      if (cap->norm) put_row(cap->norm + (size_t)rows[q] * N, q < n_normrows ? o_norm + es * N * q : o_raw + es * N * q);
    }
    if (cap->total) put_row(cap->total, o_tot);
  }
  ctx->last_path = 6;
  return KSG_OK;
}

int eval_internal(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods) return fail(ctx, KSG_E_INVALID, "pod index");
  if ((rc = check_blobs(ctx, pod, 1))) return rc;
  if (eval_fast_eligible(ctx, pod)) return eval_fast(ctx, pod, res, cap);   // consumes or flushes a staged append
  if ((rc = srv_stop(ctx))) return rc;   // the other paths put work on the stream
  if (eval_topo_eligible(ctx, pod)) return eval_topo_fast(ctx, pod, res, cap);
  int32_t pl;
  return run_internal(ctx, pod, 1, 0, &pl, res, cap);
}

// Grow a device array to `need` elements, keeping its first `used` ones.
template <typename T>
int dgrow(ksg_ctx* ctx, T** p, size_t* cap, size_t used, size_t need) {
  if (need <= *cap && *p) return KSG_OK;
  if (int rc = srv_stop(ctx)) return rc;
  const size_t ncap = std::max(need, 2 * *cap);
  T* np = nullptr;
  int rc = dalloc(ctx, &np, ncap);
  if (rc) return rc;
  if (used && *p) HIPC(ctx, hipMemcpyAsync(np, *p, used * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  if (*p) {
    auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), (void*)*p);
    if (it != ctx->allocs.end()) ctx->allocs.erase(it);
    (void)hipFree(*p);
  }
  *p = np;
  *cap = ncap;
  return KSG_OK;
}

// Every program offset of a pod lies inside its blob (the kernels index them
// relative to the staged blob), the blob inside the pool of `len` words.
bool pod_offsets_ok(const ksg_pod& p, int64_t len) {
  if (p.blob < 0 || p.blob_len < 0 || (int64_t)p.blob + p.blob_len > len) return false;
  for (int32_t off : {p.tol, p.na_req, p.na_pref, p.img, p.pts, p.ipa, p.commit, p.ports, p.vol})
    if (off >= 0 && (off < p.blob || off >= p.blob + p.blob_len)) return false;
  return true;
}

// The pod's ports program (n_conf conf[] n_own own[]) lies inside its blob
// and names only UsedPorts bits that exist (< 32 * PW): the kernels index the
// per-node bitmap with these ids.  `at` reads a program word.
template <class At>
bool ports_prog_ok(const ksg_pod& p, int PW, At at) {
  if (p.ports < 0) return true;
  const int64_t end = (int64_t)p.blob + p.blob_len;
  int64_t w = p.ports;
  for (int part = 0; part < 2; part++) {
    if (w >= end) return false;
    const int64_t n = at(w++);
    if (n < 0 || w + n > end) return false;
    for (int64_t i = 0; i < n; i++) {
      const int64_t id = at(w++);
      if (id < 0 || id >= 32 * (int64_t)PW) return false;
    }
  }
  return true;
}

// Extent of the program words a pod uses (blob and node set).
int64_t pod_prog_end(const ksg_pod& p, int N) {
  int64_t e = (int64_t)p.blob + p.blob_len;
  if (p.node_set >= 0) e = std::max<int64_t>(e, (int64_t)p.node_set + (N + 31) / 32);
  return e;
}

int32_t na_pref_weight_sum(const std::vector<int32_t>& prog, const ksg_pod& p);

// Issue a pending staged append (append_internal) as two stream-ordered
// copies.  Every entry point that launches kernels reading d_pods / d_prog
// calls this first, except the per-cycle evaluation of the staged pod.
// One assume (sign 1) or its removal (-1) on the stream: the record and the
// commit program by value when they fit CommitArgs, else read by the kernel.
int launch_commit(ksg_ctx* ctx, int32_t pod, int32_t node, int sign) {
  const ksg_pod& p = ctx->h_pods[pod];
  CommitArgs k{};
  k.node = node;
  k.sign = sign;
  for (int r = 0; r < KSG_MAX_RES; r++) k.req[r] = p.req[r];
  k.nz_cpu = p.nz_cpu;
  k.nz_mem = p.nz_mem;
  k.ports = p.ports >= 0 ? ctx->d_prog + p.ports : nullptr;
  bool inl = true;   // the commit program by value when it fits the arguments
  if (p.commit >= 0) {
    const int32_t* w = ctx->h_prog.data() + p.commit;
    k.ns = w[0];
    k.nt = w[1 + k.ns];
    inl = inl && k.ns <= kCommitSel && k.nt <= kCommitTmpl;
    if (inl) {
      for (int i = 0; i < k.ns; i++) k.sel[i] = w[1 + i];
      for (int i = 0; i < k.nt; i++) {
        k.tm[i] = w[2 + k.ns + 2 * i];
        k.tw[i] = w[3 + k.ns + 2 * i];
      }
    }
  }
  if (inl)
    hipLaunchKernelGGL(ksg_commit_args_kernel, dim3(1), dim3(64), 0, ctx->stream, ctx->c, ctx->st, k, ctx->pct,
                       ctx->pct_valid ? 1 : 0);
  else
    hipLaunchKernelGGL(ksg_commit_kernel, dim3(1), dim3(64), 0, ctx->stream, ctx->c, ctx->st, ctx->d_pods,
                       ctx->d_prog, pod, node, sign, ctx->pct, ctx->pct_valid ? 1 : 0);
  HIPC(ctx, hipGetLastError());
  return KSG_OK;
}

int flush_stage(ksg_ctx* ctx) {
  if (!ctx->stage_pending) return KSG_OK;
  if (int rc = srv_stop(ctx)) return rc;
  const size_t pb = sizeof(ksg_pod) * ctx->stage_n, gb = sizeof(int32_t) * ctx->stage_len;
  if (pb)
    HIPC(ctx, hipMemcpyAsync(ctx->d_pods + ctx->stage_first, ctx->h_stage, pb, hipMemcpyHostToDevice, ctx->stream));
  if (gb)
    HIPC(ctx, hipMemcpyAsync(ctx->d_prog + ctx->stage_base, ctx->h_stage + pb, gb, hipMemcpyHostToDevice, ctx->stream));
  HIPC(ctx, hipEventRecord(ctx->ev_stage, ctx->stream));
  ctx->stage_pending = false;
  return KSG_OK;
}

// Launch a deferred assume (ksg_commit): every entry point that reads or
// replaces the node state calls this first, except the per-cycle evaluation,
// whose kernel applies the assume itself (ksched_cycle.h, cm_*).
int flush_commit(ksg_ctx* ctx) {
  if (ctx->pc_node < 0) return KSG_OK;
  if (int rc = srv_stop(ctx)) return rc;
  const int pod = ctx->pc_pod, node = ctx->pc_node;
  ctx->pc_node = -1;
  return launch_commit(ctx, pod, node, 1);
}

// The pod's volume program (encoder.py Encoder._volume_plan grammar) lies
// inside its blob and names only label columns < L and node indices < N:
// vol_filter (ksched_device.h) walks it without bounds checks.
template <class At>
bool vol_prog_ok(const ksg_pod& p, int L, int N, At at) {
  if (p.vol < 0) return true;
  const int64_t end = (int64_t)p.blob + p.blob_len;
  int64_t w = p.vol;
  auto take = [&](int64_t& v) {
    if (w >= end) return false;
    v = at(w++);
    return true;
  };
  auto col_ok = [&](int64_t c) { return c >= 0 && c < L; };
  auto req_ok = [&]() {   // col op n values
    int64_t col, op, n;
    if (!take(col) || !take(op) || !take(n) || n < 0 || w + n > end) return false;
    if (op != 6 && !col_ok(col)) return false;
    w += n;
    return true;
  };
  auto terms_ok = [&](int64_t nt) {
    for (int64_t t = 0; t < nt; t++) {
      int64_t nr;
      if (!take(nr) || nr < 0) return false;
      for (int64_t r = 0; r < nr; r++)
        if (!req_ok()) return false;
    }
    return true;
  };
  int64_t flags, nb, np, nz;
  if (!take(flags) || !take(nb) || nb < 0) return false;
  for (int64_t b = 0; b < nb; b++) {
    int64_t kind, nt;
    if (!take(kind)) return false;
    if (kind == 0) continue;
    if (kind != 1 || !take(nt) || nt < -1 || !terms_ok(nt)) return false;
  }
  if (!take(np) || np < 0) return false;
  for (int64_t k = 0; k < np; k++) {
    int64_t sel, nt;
    if (!take(sel) || sel < -2 || sel >= N || !take(nt) || nt < -1 || !terms_ok(nt)) return false;
  }
  for (int k = 0; k < 4; k++) {
    int64_t c;
    if (!take(c) || (c != -1 && !col_ok(c))) return false;
  }
  if (!take(nz) || nz < 0) return false;
  for (int64_t k = 0; k < nz; k++) {
    int64_t col, gcol, n;
    if (!take(col) || !take(gcol) || !col_ok(col) || !col_ok(gcol)) return false;
    for (int part = 0; part < 2; part++) {
      if (!take(n) || n < 0 || w + n > end) return false;
      w += n;
    }
  }
  return true;
}

// An assume the per-cycle kernel can apply: node columns only (no selector
// counts, template tables or host ports).
bool commit_deferrable(const ksg_ctx* ctx, int32_t pod) {
  const ksg_pod& p = ctx->h_pods[pod];
  if (p.ports >= 0) return false;
  if (p.commit < 0) return true;
  const int32_t* w = ctx->h_prog.data() + p.commit;
  return w[0] == 0 && w[1] == 0;
}

int append_internal(ksg_ctx* ctx, const ksg_pod* pods, int32_t n, const int32_t* prog, int64_t prog_len,
                    int64_t prog_base) {
  if (!ctx->have_wl) return fail(ctx, KSG_E_STATE, "load a workload before appending");
  if (n < 0 || prog_len < 0 || (n > 0 && !pods) || (prog_len > 0 && !prog)) return fail(ctx, KSG_E_INVALID, "append arguments");
  if (prog_base < ctx->prog_used || prog_base > (int64_t)ctx->h_prog.size())
    return fail(ctx, KSG_E_INVALID, "append: prog_base cuts into loaded programs or leaves a gap");
  const int64_t new_len = prog_base + prog_len;
  const int N = ctx->c.N;
  int64_t used = ctx->prog_used;
  int32_t max_blob = ctx->max_blob;
  for (int i = 0; i < n; i++) {
    const ksg_pod& p = pods[i];
    if (p.blob < 0 || p.blob_len < 0 || pod_prog_end(p, N) > new_len || !pod_offsets_ok(p, new_len))
      return fail(ctx, KSG_E_INVALID, "appended pod program outside the pool");
    if (!ports_prog_ok(p, ctx->c.PW, [&](int64_t k) -> int64_t {
          return k >= prog_base ? prog[k - prog_base] : ctx->h_prog[k];
        }))
      return fail(ctx, KSG_E_INVALID, "appended pod: host-port ids outside the vocabulary");
    if (!vol_prog_ok(p, ctx->c.L, N, [&](int64_t k) -> int64_t {
          return k >= prog_base ? prog[k - prog_base] : ctx->h_prog[k];
        }))
      return fail(ctx, KSG_E_INVALID, "appended pod: malformed volume program");
    used = std::max(used, pod_prog_end(p, N));
    max_blob = std::max(max_blob, p.blob_len);
  }
  HIPC(ctx, hipSetDevice(ctx->device));
  int rc;
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = dgrow(ctx, &ctx->d_pods, &ctx->pod_cap, (size_t)ctx->n_pods, (size_t)ctx->n_pods + n))) return rc;
  if ((rc = dgrow(ctx, &ctx->d_prog, &ctx->prog_cap, (size_t)prog_base, (size_t)std::max<int64_t>(new_len, 1)))) return rc;
  const size_t pb = sizeof(ksg_pod) * n, gb = sizeof(int32_t) * prog_len;
  if (pb + gb <= (1u << 20)) {
    // the per-cycle append: into a pinned, fine-grained staging buffer, no
    // host wait and no copy launch (the caller's buffers are free once this
    // returns).  The copy to the device arrays is pending: the next ksg_eval
    // of the pod consumes it (ksg_capture_eval reads the staged words and its
    // first workgroup writes them to d_pods / d_prog), any other call issues
    // it first (flush_stage).
    if (!ctx->ev_stage) HIPC(ctx, hipEventCreateWithFlags(&ctx->ev_stage, hipEventDisableTiming));
    else HIPC(ctx, hipEventSynchronize(ctx->ev_stage));   // a flushed copy has left the buffer
    if (pb + gb > ctx->h_stage_bytes) {
      if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_mb) {
    if (ctx->mb_device) (void)hipFree(ctx->mb_alloc);
    else (void)hipHostFree(ctx->h_mb);
  }
      ctx->h_stage = nullptr;
      ctx->d_stage = nullptr;
      ctx->h_stage_bytes = 0;
      HIPC(ctx, hipHostMalloc((void**)&ctx->h_stage, 1u << 20, hipHostMallocMapped | hipHostMallocCoherent));
      ctx->h_stage_bytes = 1u << 20;
      void* dp = nullptr;
      HIPC(ctx, hipHostGetDevicePointer(&dp, ctx->h_stage, 0));
      ctx->d_stage = static_cast<const char*>(dp);
    }
    if (pb) std::memcpy(ctx->h_stage, pods, pb);
    if (gb) std::memcpy(ctx->h_stage + pb, prog, gb);
    ctx->stage_pending = true;
    ctx->stage_first = ctx->n_pods;
    ctx->stage_n = n;
    ctx->stage_base = prog_base;
    ctx->stage_len = prog_len;
  } else {
    if ((rc = srv_stop(ctx))) return rc;
    if (n) HIPC(ctx, hipMemcpyAsync(ctx->d_pods + ctx->n_pods, pods, pb, hipMemcpyHostToDevice, ctx->stream));
    if (prog_len) HIPC(ctx, hipMemcpyAsync(ctx->d_prog + prog_base, prog, gb, hipMemcpyHostToDevice, ctx->stream));
    HIPC(ctx, hipStreamSynchronize(ctx->stream));
  }
  ctx->h_prog.resize(new_len);
  if (prog_len) std::copy(prog, prog + prog_len, ctx->h_prog.begin() + prog_base);
  for (int i = 0; i < n; i++) {
    ctx->h_pods.push_back(pods[i]);
    ctx->h_na_pref_sum.push_back(na_pref_weight_sum(ctx->h_prog, pods[i]));
  }
  ctx->n_pods += n;
  ctx->prog_used = used;
  ctx->max_blob = max_blob;
  return KSG_OK;
}

// Existing pods' required anti-affinity templates matching the preemptor
// (the m_anti list of its InterPodAffinity program, parse_topo's layout);
// bounds-checked against the host pool, INT32_MAX when malformed.
int32_t preempt_n_ma(const ksg_ctx* ctx, const ksg_pod& p) {
  if (p.ipa < 0) return 0;
  const std::vector<int32_t>& P = ctx->h_prog;
  const int64_t end = std::min<int64_t>((int64_t)p.blob + p.blob_len, (int64_t)P.size());
  int64_t w = p.ipa;
  auto at = [&](int64_t i) -> int64_t { return i >= 0 && i < end ? P[i] : -1; };
  const int64_t na = at(w);
  if (na < 0) return 0x7fffffff;
  w += 3 + na;
  const int64_t nn = at(w++);
  if (nn < 0) return 0x7fffffff;
  w += 2 * nn;
  const int64_t np = at(w++);
  if (np < 0) return 0x7fffffff;
  w += 3 * np;
  const int64_t nm = at(w);
  return nm < 0 ? 0x7fffffff : (int32_t)nm;
}

int32_t na_pref_weight_sum(const std::vector<int32_t>& prog, const ksg_pod& p) {
  // na_pref := n_terms { weight n_reqs requirement[n_reqs] }; every word read
  // is bounds-checked against the pod's blob (a malformed program yields
  // INT32_MAX, which keeps the pod off the batched path)
  const int64_t off = p.na_pref;
  if (off < 0) return 0;
  const int64_t end = std::min<int64_t>((int64_t)p.blob + p.blob_len, (int64_t)prog.size());
  int64_t w = off;
  auto at = [&](int64_t i, bool& ok) -> int64_t {
    if (i < 0 || i >= end) { ok = false; return 0; }
    return prog[i];
  };
  bool ok = true;
  const int64_t nt = at(w++, ok);
  int64_t s = 0;
  for (int64_t t = 0; ok && t < nt; t++) {
    s += at(w++, ok);
    const int64_t nr = at(w++, ok);
    for (int64_t r = 0; ok && r < nr; r++) {
      const int64_t nv = at(w + 2, ok);
      if (nv < 0) ok = false;
      w += 3 + nv;
    }
  }
  if (!ok || s < 0) return 0x7fffffff;
  return s > 0x7fffffff ? 0x7fffffff : (int32_t)s;
}

}  // namespace

extern "C" {

int ksg_abi_version(void) { return KSG_ABI_VERSION; }

int ksg_open(int device, ksg_ctx** out) {
  if (!out) return KSG_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KSG_E_DEVICE;
  if (device < 0 || device >= ndev) return KSG_E_INVALID;
  ksg_ctx* ctx = new ksg_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return KSG_E_DEVICE;
  }
  if (const char* f = getenv("KSG_FORCE_PATH")) ctx->force_path = atoi(f);
  if (const char* f = getenv("KSG_TOPO_COOP")) ctx->topo_coop = atoi(f) != 0;
  if (const char* f = getenv("KSG_TOPO_WINDOW")) ctx->topo_window = atoi(f) != 0;
  if (const char* f = getenv("KSG_TOPO_WINDOW_K")) ctx->win_kmax = std::max(1, std::min(atoi(f), kWinMax));
  if (const char* f = getenv("KSG_COOP_PMODE")) ctx->coop_pmode = atoi(f) != 0;
  if (const char* f = getenv("KSG_COOP_TABLES")) ctx->coop_tables = atoi(f) != 0;
  if (const char* f = getenv("KSG_DEFER_COMMIT")) ctx->defer_commit = atoi(f) != 0;
  if (const char* f = getenv("KSG_BATCH_MODE")) {
    const std::string m(f);
    ctx->batch_mode = m == "slot" ? 2 : m == "window" ? 4 : 6;
  }
  if (const char* f = getenv("KSG_PIPE_WINDOW")) ctx->pipe_window = atoi(f) != 0;
  if (const char* f = getenv("KSG_PIPE_OVERLAP")) ctx->pipe_overlap = atoi(f) != 0;
  if (const char* f = getenv("KSG_SPEC_PERSIST")) ctx->spec_persist = atoi(f) != 0;
  if (const char* f = getenv("KSG_EVAL_FAST")) ctx->eval_fast = atoi(f) != 0;
  if (const char* f = getenv("KSG_CYCLE_COOP")) ctx->cycle_coop = atoi(f) != 0;
  if (const char* f = getenv("KSG_COOP_LAUNCH")) ctx->coop_launch = ctx->topo_eval_coop = atoi(f) != 0;
  if (const char* f = getenv("KSG_PC_TABLES")) ctx->pc_tables = atoi(f) != 0;
  if (const char* f = getenv("KSG_CYCLE_SYS")) ctx->cycle_sys = atoi(f) != 0;
  if (const char* f = getenv("KSG_CYCLE_SERVER")) ctx->srv_mode = atoi(f) != 0;
  if (const char* f = getenv("KSG_CYCLE_KN")) {
    const int v = atoi(f);
    ctx->cycle_kn = v >= 4 ? 4 : v >= 2 ? 2 : 1;
  }
  if (const char* f = getenv("KSG_TEST_INJECT_WALK_ERR")) ctx->inject_walk_err = atoi(f) != 0;
  if (const char* f = getenv("KSG_TEST_INJECT_TIMEOUT")) ctx->inject_timeout = atoi(f);
  if (const char* f = getenv("KSG_SLOT_BLOCK")) {
    const int v = atoi(f);
    ctx->slot_block = v <= 64 ? 64 : 128;
  }
  *out = ctx;
  return KSG_OK;
}

int ksg_close(ksg_ctx* ctx) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx) return KSG_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  free_all(ctx);
  for (hipEvent_t e : ctx->tev) (void)hipEventDestroy(e);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  for (int q = 0; q < 2; q++) {
    if (ctx->ev_tk[q]) (void)hipEventDestroy(ctx->ev_tk[q]);
    if (ctx->ev_p2[q]) (void)hipEventDestroy(ctx->ev_p2[q]);
  }
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->h_ev) (void)hipHostFree(ctx->h_ev);
  if (ctx->h_p2done) (void)hipHostFree(ctx->h_p2done);
  if (ctx->h_evt) (void)hipHostFree(ctx->h_evt);
  if (ctx->d_json_tab) (void)hipFree(ctx->d_json_tab);
  if (ctx->json_stream) (void)hipStreamSynchronize(ctx->json_stream);
  for (int q = 0; q < ksg_ctx::kJsonSlots; q++) {
    if (ctx->d_json_out[q]) (void)hipFree(ctx->d_json_out[q]);
    if (ctx->h_json[q]) (void)hipHostFree(ctx->h_json[q]);
    if (ctx->json_copied[q]) (void)hipEventDestroy(ctx->json_copied[q]);
  }
  if (ctx->json_written) (void)hipEventDestroy(ctx->json_written);
  if (ctx->json_stream) (void)hipStreamDestroy(ctx->json_stream);
  if (ctx->d_json_err) (void)hipFree(ctx->d_json_err);
  if (ctx->h_json_err) (void)hipHostFree(ctx->h_json_err);
  if (ctx->d_json_scratch) (void)hipFree(ctx->d_json_scratch);
  if (ctx->d_json_arena) (void)hipFree(ctx->d_json_arena);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->ev_stage) (void)hipEventDestroy(ctx->ev_stage);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return KSG_OK;
}

const char* ksg_last_error(ksg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ksg_set_profile(ksg_ctx* ctx, const ksg_profile* prof) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !prof) return KSG_E_INVALID;
  if (prof->n_filter < 0 || prof->n_filter > KSG_NPLUGINS || prof->fit_n < 0 || prof->fit_n > KSG_MAX_RES ||
      prof->ba_n < 0 || prof->ba_n > KSG_MAX_RES || prof->fit_strategy < KSG_LEAST_ALLOCATED ||
      prof->fit_strategy > KSG_REQUESTED_TO_CAPACITY_RATIO || prof->shape_n < 0 || prof->shape_n > KSG_MAX_SHAPE ||
      (prof->fit_strategy == KSG_REQUESTED_TO_CAPACITY_RATIO && prof->shape_n == 0))
    return fail(ctx, KSG_E_INVALID, "profile field out of range");
  for (int i = 0; i < prof->shape_n; i++)   // ValidateNodeResourcesFitArgs' shape rules (scores already x 10)
    if (prof->shape_util[i] < 0 || prof->shape_util[i] > 100 || prof->shape_score[i] < 0 ||
        prof->shape_score[i] > 100 || (i > 0 && prof->shape_util[i] <= prof->shape_util[i - 1]))
      return fail(ctx, KSG_E_INVALID, "RequestedToCapacityRatio shape out of range or not increasing");
  ctx->prof = *prof;
  ctx->have_prof = true;
  ctx->ev_prof_dirty = true;
  return KSG_OK;
}

int ksg_load_nodes(ksg_ctx* ctx, const ksg_nodes* nd, const ksg_topology* tp) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !nd || !tp) return KSG_E_INVALID;
  HIPC(ctx, hipSetDevice(ctx->device));
  if (nd->n_nodes <= 0 || nd->n_res < 3 || nd->n_res > KSG_MAX_RES)
    return fail(ctx, KSG_E_INVALID, "bad node table sizes");
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  free_all(ctx);
  ctx->have_nodes = ctx->have_wl = false;
  const int N = nd->n_nodes, R = nd->n_res, L = std::max(nd->n_label_cols, 1);
  DevCluster& c = ctx->c;
  c = DevCluster{};
  c.N = N; c.R = R; c.L = nd->n_label_cols; c.T = nd->max_taints; c.I = nd->max_images;
  c.V = nd->n_taint_vocab; c.W = std::max(1, (nd->n_taint_vocab + 31) / 32);
  if (nd->n_port_vocab < 0) return fail(ctx, KSG_E_INVALID, "bad host-port vocabulary size");
  c.PW = std::max(1, (nd->n_port_vocab + 31) / 32);
  c.lab_stride = N;
  c.lab_base = 0;
  int rc = 0;
#define UP(field, src, cnt) if ((rc = upc(ctx, c.field, src, cnt))) return rc
  UP(alloc, nd->alloc, (size_t)R * N);
  UP(allowed, nd->allowed_pods, N);
  UP(unsched, nd->unschedulable, N);
  UP(label_val, nd->label_val, (size_t)L * N);
  UP(label_num, nd->label_num, (size_t)L * N);
  UP(label_num_ok, nd->label_num_ok, (size_t)L * N);
  UP(taints, nd->taints, (size_t)c.T * N);
  UP(taint_effect, nd->taint_effect, (size_t)std::max(c.V, 1));
  UP(images, nd->images, (size_t)c.I * N);
  {
    float2* r32;
    double2* r64;
    if ((rc = dalloc(ctx, &r32, N))) return rc;
    if ((rc = dalloc(ctx, &r64, N))) return rc;
    c.rcp32 = r32;
    c.rcp64 = r64;
    if (R > KSG_RES_MEM && N > 0) {
      hipLaunchKernelGGL(ksg_node_rcp, dim3((N + 255) / 256), dim3(256), 0, ctx->stream, c, r32, r64);
      HIPC(ctx, hipGetLastError());
    }
  }
  c.S = tp->n_selectors;
  c.n_tmpl = tp->n_templates;
  const int nt = std::max(tp->n_templates, 1);
  UP(tmpl_col, tp->tmpl_col, nt);
  UP(tmpl_kind, tp->tmpl_kind, nt);
  UP(tmpl_weight, tp->tmpl_weight, nt);
  UP(col_vocab, tp->col_vocab, L);
  UP(col_unique, tp->col_unique, L);
  ctx->h_col_vocab.assign(tp->col_vocab, tp->col_vocab + L);
  ctx->h_col_unique.assign(tp->col_unique, tp->col_unique + L);
  UP(log_table, tp->log_table, tp->log_n);
  c.log_n = tp->log_n;
  std::vector<int32_t> off(nt, 0);
  size_t total = 0;
  for (int t = 0; t < tp->n_templates; t++) {
    off[t] = (int32_t)total;
    total += (size_t)std::max(tp->col_vocab[tp->tmpl_col[t]], 1);
  }
  ctx->tab_words = std::max<size_t>(total, 1);
  UP(tmpl_off, off.data(), nt);
#undef UP
  DevState& st = ctx->st;
  st = DevState{};
  if ((rc = upload(ctx, &st.requested, nd->requested, (size_t)R * N))) return rc;
  if ((rc = upload(ctx, &st.nonzero, nd->nonzero, (size_t)2 * N))) return rc;
  if ((rc = upload(ctx, &st.pod_count, nd->pod_count, N))) return rc;
  if ((rc = dalloc(ctx, &st.cnt, (size_t)std::max(c.S, 1) * N))) return rc;
  if ((rc = dalloc(ctx, &st.tab, ctx->tab_words))) return rc;
  if ((rc = dalloc(ctx, &st.tmpl_total, nt))) return rc;
  if ((rc = dalloc(ctx, &st.partial, N))) return rc;
  if ((rc = dalloc(ctx, &st.sraw, (size_t)4 * N))) return rc;
  if ((rc = dalloc(ctx, &st.ports, (size_t)c.PW * N))) return rc;   // UsedPorts: empty at load
  HIPC(ctx, hipMemsetAsync(st.ports, 0, sizeof(uint32_t) * c.PW * (size_t)N, ctx->stream));
  HIPC(ctx, hipMemsetAsync(st.cnt, 0, sizeof(int32_t) * std::max(c.S, 1) * (size_t)N, ctx->stream));
  HIPC(ctx, hipMemsetAsync(st.tab, 0, sizeof(int32_t) * ctx->tab_words, ctx->stream));
  HIPC(ctx, hipMemsetAsync(st.tmpl_total, 0, sizeof(int32_t) * nt, ctx->stream));
  if ((rc = upload(ctx, &ctx->d_req0, nd->requested, (size_t)R * N))) return rc;
  if ((rc = upload(ctx, &ctx->d_nz0, nd->nonzero, (size_t)2 * N))) return rc;
  if ((rc = upload(ctx, &ctx->d_pc0, nd->pod_count, N))) return rc;
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  ctx->have_nodes = true;
  return KSG_OK;
}

int ksg_load_workload(ksg_ctx* ctx, const ksg_workload* wl) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !wl || (!wl->pods && wl->n_pods > 0) || wl->n_pods < 0 || wl->prog_len < 0 ||
      (!wl->prog && wl->prog_len > 0))
    return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "load nodes before the workload");
  HIPC(ctx, hipSetDevice(ctx->device));
  {   // a deferred assume reads its pod from the pool about to be replaced
    const int rc = flush_commit(ctx);
    if (rc) return rc;
  }
  ctx->pct_valid = false;
  ctx->stage_pending = false;   // a staged append of the replaced workload
  ctx->h_pods.assign(wl->pods, wl->pods + wl->n_pods);
  std::vector<int32_t> prog(wl->prog, wl->prog + wl->prog_len);
  ctx->max_blob = 0;
  ctx->h_na_pref_sum.assign(wl->n_pods, 0);
  for (int i = 0; i < wl->n_pods; i++) {
    const ksg_pod& p = ctx->h_pods[i];
    ctx->max_blob = std::max(ctx->max_blob, p.blob_len);
    if (!pod_offsets_ok(p, wl->prog_len)) return fail(ctx, KSG_E_INVALID, "pod program outside its blob / the pool");
    if (!ports_prog_ok(p, ctx->c.PW, [&](int64_t k) -> int64_t { return prog[k]; }))
      return fail(ctx, KSG_E_INVALID, "pod " + std::to_string(i) + ": host-port ids outside the vocabulary");
    if (!vol_prog_ok(p, ctx->c.L, ctx->c.N, [&](int64_t k) -> int64_t { return prog[k]; }))
      return fail(ctx, KSG_E_INVALID, "pod " + std::to_string(i) + ": malformed volume program");
    if (p.node_set >= 0 && (int64_t)p.node_set + (ctx->c.N + 31) / 32 > wl->prog_len)
      return fail(ctx, KSG_E_INVALID, "node set outside the program pool");
    ctx->h_na_pref_sum[i] = na_pref_weight_sum(prog, p);
  }
  ctx->h_prog = std::move(prog);
  ctx->prog_used = 0;
  for (int i = 0; i < wl->n_pods; i++) ctx->prog_used = std::max(ctx->prog_used, pod_prog_end(ctx->h_pods[i], ctx->c.N));
  int rc;
  if (ctx->d_pods) {   // a reload: drop the previous workload's buffers
    for (void* q : {(void*)ctx->d_pods, (void*)ctx->d_prog}) {
      auto it = std::find(ctx->allocs.begin(), ctx->allocs.end(), q);
      if (it != ctx->allocs.end()) ctx->allocs.erase(it);
      (void)hipFree(q);
    }
    ctx->d_pods = nullptr;
    ctx->d_prog = nullptr;
  }
  // an empty workload (pods arrive later through ksg_append_pods) still gets
  // one-element buffers
  if ((rc = wl->n_pods ? upload(ctx, &ctx->d_pods, wl->pods, wl->n_pods) : dalloc(ctx, &ctx->d_pods, 1))) return rc;
  if ((rc = wl->prog_len ? upload(ctx, &ctx->d_prog, wl->prog, (size_t)wl->prog_len) : dalloc(ctx, &ctx->d_prog, 1)))
    return rc;
  ctx->pod_cap = std::max(wl->n_pods, 1);
  ctx->prog_cap = (size_t)std::max<int64_t>(wl->prog_len, 1);
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_pods = wl->n_pods;
  ctx->have_wl = true;
  return KSG_OK;
}

int ksg_eval(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_capture* cap) {
  if (!res) return fail(ctx, KSG_E_INVALID, "null result");
  return eval_internal(ctx, pod, res, cap);
}

int ksg_eval_view(ksg_ctx* ctx, int32_t pod, ksg_result* res, ksg_eval_rows* rows) {
  if (!ctx || !res || !rows) return ctx ? fail(ctx, KSG_E_INVALID, "null result") : KSG_E_INVALID;
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods) return fail(ctx, KSG_E_INVALID, "pod index");
  if ((rc = check_blobs(ctx, pod, 1))) return rc;
  if (eval_fast_eligible(ctx, pod)) return eval_fast(ctx, pod, res, nullptr, rows);
  if ((rc = srv_stop(ctx))) return rc;   // the other paths put work on the stream
  if (eval_topo_eligible(ctx, pod)) return eval_topo_fast(ctx, pod, res, nullptr, rows);
  // otherwise: run_internal into library-owned int64 rows
  const size_t N = ctx->c.N;
  ctx->view_fs.resize(N);
  ctx->view_rows.resize((2 * (size_t)KSG_NPLUGINS + 1) * N);
  ksg_capture cap{ctx->view_fs.data(), ctx->view_rows.data(), ctx->view_rows.data() + KSG_NPLUGINS * N,
                  ctx->view_rows.data() + 2 * KSG_NPLUGINS * N};
  int32_t pl;
  if ((rc = run_internal(ctx, pod, 1, 0, &pl, res, &cap))) return rc;
  *rows = ksg_eval_rows{};
  rows->n_nodes = (int32_t)N;
  rows->elem_bytes = 8;
  rows->fstatus = cap.fstatus;
  for (int p = 0; p < KSG_NPLUGINS; p++)
    if ((ctx->prof.score_mask >> p) & 1u) {
      rows->raw[p] = cap.raw + (size_t)p * N;
      rows->norm[p] = cap.norm + (size_t)p * N;
    }
  rows->total = cap.total;
  return KSG_OK;
}

int ksg_append_pods(ksg_ctx* ctx, const ksg_workload* tail, int64_t prog_base) {
  if (!ctx || !tail) return KSG_E_INVALID;
  return append_internal(ctx, tail->pods, tail->n_pods, tail->prog, tail->prog_len, prog_base);
}

int ksg_eval_pod(ksg_ctx* ctx, const ksg_pod* pod, const int32_t* prog, int64_t prog_len, ksg_result* res,
                 ksg_capture* cap) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !pod || !res) return KSG_E_INVALID;
  if (!ctx->have_wl) return fail(ctx, KSG_E_STATE, "load a workload first");
  // Stage the pod behind the loaded workload (offsets rebased), evaluate it,
  // then drop it again: the device buffers keep the capacity.
  const int64_t base = (int64_t)ctx->h_prog.size();
  ksg_pod p = *pod;
  for (int32_t* f : {&p.tol, &p.na_req, &p.na_pref, &p.img, &p.node_set, &p.pts, &p.ipa, &p.commit, &p.blob,
                     &p.ports, &p.vol})
    if (*f >= 0) *f = (int32_t)(*f + base);
  const int32_t n0 = ctx->n_pods, blob0 = ctx->max_blob;
  const int64_t used0 = ctx->prog_used;
  int rc = append_internal(ctx, &p, 1, prog, prog_len, base);
  if (!rc) rc = eval_internal(ctx, n0, res, cap);
  if (ctx->stage_pending && ctx->stage_first >= n0) ctx->stage_pending = false;   // the staged pod is dropped
  if (ctx->n_pods > n0) {
    ctx->n_pods = n0;
    ctx->h_pods.resize(n0);
    ctx->h_na_pref_sum.resize(n0);
    ctx->h_prog.resize(base);
    ctx->prog_used = used0;
    ctx->max_blob = blob0;
  }
  return rc;
}

int ksg_eval_skipping(ksg_ctx* ctx, int32_t pod, uint32_t filter_skip, ksg_result* res, ksg_capture* cap) {
  if (!ctx || !res) return ctx ? fail(ctx, KSG_E_INVALID, "null result") : KSG_E_INVALID;
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods) return fail(ctx, KSG_E_INVALID, "pod index");
  if ((rc = flush_stage(ctx)) || (rc = srv_stop(ctx))) return rc;
  // the record with the extra Skip bits, on the host (the dispatch reads it)
  // and the device; the original goes back once the evaluation has synced
  const ksg_pod keep = ctx->h_pods[pod];
  ctx->h_pods[pod].filter_skip |= filter_skip;
  HIPC(ctx, hipMemcpyAsync(ctx->d_pods + pod, &ctx->h_pods[pod], sizeof(ksg_pod), hipMemcpyHostToDevice,
                           ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  rc = eval_internal(ctx, pod, res, cap);
  int rc2 = srv_stop(ctx);
  ctx->h_pods[pod] = keep;
  HIPC(ctx, hipMemcpyAsync(ctx->d_pods + pod, &ctx->h_pods[pod], sizeof(ksg_pod), hipMemcpyHostToDevice,
                           ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return rc ? rc : rc2;
}

int ksg_annotator_attach(ksg_ctx* ctx, const ksg_annotator* ann, const int64_t* weight, uint32_t normalize_mask) {
  if (int rc_ = srv_stop(ctx)) return rc_;
  if (!ctx || !ann || !weight) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "load nodes before attaching an annotator");
  JsonHostTables t;
  int rc = ksg_annotator_json_tables(ann, &t);
  if (rc) return fail(ctx, rc, "annotator tables");
  if ((int)t.node_order.size() != ctx->c.N) return fail(ctx, KSG_E_INVALID, "annotator and context node counts differ");
  if (t.max_taints != ctx->c.T && ctx->c.T > 0) return fail(ctx, KSG_E_INVALID, "annotator and context taint slots differ");
  HIPC(ctx, hipSetDevice(ctx->device));
  // one block: node key offsets (8-aligned first), then the 4-byte arrays, then the bytes
  std::vector<char> blob;
  auto put = [&](const void* p, size_t n) {
    const size_t at = (blob.size() + 7) & ~(size_t)7;
    blob.resize(at + n);
    if (n) std::memcpy(blob.data() + at, p, n);
    return at;
  };
  const size_t o_nko = put(t.node_key_off.data(), 8 * t.node_key_off.size());
  const size_t o_ord = put(t.node_order.data(), 4 * t.node_order.size());
  const size_t o_pko = put(t.plugin_key_off.data(), 4 * t.plugin_key_off.size());
  const size_t o_mo = put(t.msg_off.data(), 4 * t.msg_off.size());
  const size_t o_tmo = put(t.taint_msg_off.data(), 4 * t.taint_msg_off.size());
  const size_t o_fpo = put(t.fit_part_off.data(), 4 * t.fit_part_off.size());
  const size_t o_nk = put(t.node_keys.data(), t.node_keys.size());
  const size_t o_pk = put(t.plugin_keys.data(), t.plugin_keys.size());
  const size_t o_m = put(t.msgs.data(), t.msgs.size());
  const size_t o_tm = put(t.taint_msgs.data(), t.taint_msgs.size());
  const size_t o_fp = put(t.fit_parts.data(), t.fit_parts.size());
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->d_json_tab) (void)hipFree(ctx->d_json_tab);
  ctx->d_json_tab = nullptr;
  ctx->json_N = -1;
  HIPC(ctx, hipMalloc((void**)&ctx->d_json_tab, std::max<size_t>(blob.size(), 8)));
  HIPC(ctx, hipMemcpy(ctx->d_json_tab, blob.data(), blob.size(), hipMemcpyHostToDevice));
  char* d = ctx->d_json_tab;
  JsonTables& j = ctx->json_t;
  j.node_key_off = reinterpret_cast<const int64_t*>(d + o_nko);
  j.node_order = reinterpret_cast<const int32_t*>(d + o_ord);
  j.plugin_key_off = reinterpret_cast<const int32_t*>(d + o_pko);
  j.msg_off = reinterpret_cast<const int32_t*>(d + o_mo);
  j.taint_msg_off = reinterpret_cast<const int32_t*>(d + o_tmo);
  j.fit_part_off = reinterpret_cast<const int32_t*>(d + o_fpo);
  j.node_keys = d + o_nk;
  j.plugin_keys = d + o_pk;
  j.msgs = d + o_m;
  j.taint_msgs = d + o_tm;
  j.fit_parts = d + o_fp;
  for (int i = 0; i < KSG_NPLUGINS; i++) j.by_name[i] = t.by_name[i];
  j.n_res = t.n_res;
  j.n_taint_vocab = t.n_taint_vocab;
  for (int p = 0; p < KSG_NPLUGINS; p++) ctx->json_w[p] = weight[p];
  ctx->json_norm = normalize_mask;
  ctx->json_N = ctx->c.N;
  return KSG_OK;
}

int ksg_run_queue_json_async(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                             int32_t* ticket) {
  if (!ctx || !ticket) return KSG_E_INVALID;
  if (count <= 0) return fail(ctx, KSG_E_INVALID, "ksg_run_queue_json: empty pod range");
  ctx->json_want = true;
  const int rc = run_internal(ctx, first, count, 1, placements, results, nullptr);
  ctx->json_want = false;
  if (rc) return rc;
  *ticket = ctx->json_last;
  return KSG_OK;
}

int ksg_json_wait(ksg_ctx* ctx, int32_t ticket, const char** json, const int64_t** offsets) {
  if (!ctx || !json || !offsets || ticket < 0 || ticket >= ksg_ctx::kJsonSlots || !ctx->h_json[ticket])
    return KSG_E_INVALID;
  HIPC(ctx, hipEventSynchronize(ctx->json_copied[ticket]));
  if (ctx->h_json_err[ticket]) return fail(ctx, KSG_E_INVALID, "ksg_run_queue_json: a status word without a message");
  const size_t total = (size_t)ctx->json_off[ticket].back();
  ctx->h_json[ticket][total] = 0;
  *json = ctx->h_json[ticket];
  *offsets = ctx->json_off[ticket].data();
  return KSG_OK;
}

int ksg_run_queue_json(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                       const char** json, const int64_t** offsets) {
  if (!ctx || !json || !offsets) return KSG_E_INVALID;
  if (count == 0) {
    static const char kEmpty[1] = {0};
    static const int64_t kZero[1] = {0};
    *json = kEmpty;
    *offsets = kZero;
    return KSG_OK;
  }
  int32_t t = -1;
  const int rc = ksg_run_queue_json_async(ctx, first, count, placements, results, &t);
  return rc ? rc : ksg_json_wait(ctx, t, json, offsets);
}

int ksg_run_queue(ksg_ctx* ctx, int32_t first, int32_t count, int32_t* placements, ksg_result* results,
                  ksg_capture* cap) {
  return run_internal(ctx, first, count, 1, placements, results, cap);
}

static int commit_signed(ksg_ctx* ctx, int32_t pod, int32_t node, int sign) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods || node < 0 || node >= ctx->c.N) return fail(ctx, KSG_E_INVALID, "commit range");
  HIPC(ctx, hipSetDevice(ctx->device));
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;   // one deferred assume at a time, in call order
  if (sign > 0 && ctx->defer_commit && ctx->eval_fast && commit_deferrable(ctx, pod)) {
    ctx->pc_pod = pod;   // the next per-cycle kernel applies it (or flush_commit launches it)
    ctx->pc_node = node;
    return KSG_OK;
  }
  if ((rc = srv_stop(ctx))) return rc;
  if ((rc = launch_commit(ctx, pod, node, sign))) return rc;
  // stream-ordered: the next evaluation on ctx->stream sees the update, and
  // every read-back synchronises the stream; no host wait per assume
  HIPC(ctx, hipGetLastError());
  return KSG_OK;
}

int ksg_commit(ksg_ctx* ctx, int32_t pod, int32_t node) { return commit_signed(ctx, pod, node, 1); }

int ksg_commit_batch(ksg_ctx* ctx, const int32_t* pods, const int32_t* nodes, int32_t n) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!pods || !nodes))) return fail(ctx, KSG_E_INVALID, "commit batch arguments");
  for (int32_t i = 0; i < n; i++)
    if (pods[i] < 0 || pods[i] >= ctx->n_pods || nodes[i] < 0 || nodes[i] >= ctx->c.N)
      return fail(ctx, KSG_E_INVALID, "commit batch: pod or node out of range");
  if (n == 0) return KSG_OK;
  ctx->pct_valid = false;   // the bulk bindings move the counts without the per-cycle tables
  HIPC(ctx, hipSetDevice(ctx->device));
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;
  Tmp tmp;
  int32_t *dp = nullptr, *dn = nullptr;
  TA(tmp, &dp, sizeof(int32_t) * (size_t)n);
  TA(tmp, &dn, sizeof(int32_t) * (size_t)n);
  HIPC(ctx, hipMemcpyAsync(dp, pods, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(dn, nodes, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(ksg_commit_batch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->c,
                     ctx->st, ctx->d_pods, ctx->d_prog, dp, dn, n);
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipStreamSynchronize(ctx->stream));   // the temporaries are freed on return
  return KSG_OK;
}

int ksg_uncommit(ksg_ctx* ctx, int32_t pod, int32_t node) { return commit_signed(ctx, pod, node, -1); }

int ksg_preempt_victims(ksg_ctx* ctx, int32_t pod, const int32_t* cand_node, int32_t n_cand, const int32_t* vic_off,
                        const int32_t* vic_pod, int32_t* fits, uint8_t* victim) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (pod < 0 || pod >= ctx->n_pods || n_cand < 0 || (n_cand > 0 && (!cand_node || !vic_off || !fits)))
    return fail(ctx, KSG_E_INVALID, "preempt arguments");
  if ((rc = check_blobs(ctx, pod, 1))) return rc;
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;
  if (n_cand == 0) return KSG_OK;
  const int32_t nv = vic_off[n_cand];
  if (vic_off[0] != 0 || nv < 0 || (nv > 0 && (!vic_pod || !victim)))
    return fail(ctx, KSG_E_INVALID, "preempt victim lists");
  // host-side checks of every index the kernel dereferences
  for (int k = 0; k < n_cand; k++) {
    if (cand_node[k] < 0 || cand_node[k] >= ctx->c.N) return fail(ctx, KSG_E_INVALID, "preempt candidate node");
    if (vic_off[k + 1] < vic_off[k]) return fail(ctx, KSG_E_INVALID, "preempt offsets not ascending");
  }
  for (int i = 0; i < nv; i++)
    if (vic_pod[i] < 0 || vic_pod[i] >= ctx->n_pods) return fail(ctx, KSG_E_INVALID, "preempt victim pod");
  const ksg_pod& p = ctx->h_pods[pod];
  bool fit_on = false;
  for (int kf = 0; kf < ctx->prof.n_filter; kf++) fit_on |= ctx->prof.filter_order[kf] == KSG_PL_NODE_RESOURCES_FIT;
  fit_on = fit_on && !((p.filter_skip >> KSG_PL_NODE_RESOURCES_FIT) & 1u);
  // NodePorts re-runs on the UsedPorts the removals leave (PrePorts)
  bool ports_on = false;
  for (int kf = 0; kf < ctx->prof.n_filter; kf++) ports_on |= ctx->prof.filter_order[kf] == KSG_PL_NODE_PORTS;
  ports_on = ports_on && !((p.filter_skip >> KSG_PL_NODE_PORTS) & 1u) && p.ports >= 0 && ctx->st.ports;
  if (ports_on) {
    if ((size_t)p.ports >= ctx->h_prog.size() || ctx->h_prog[p.ports] > kPreMaxConf)
      return fail(ctx, KSG_E_UNSUPPORTED, "preemption: more than " + std::to_string(kPreMaxConf) +
                                              " conflicting host-port entries for the preemptor");
  }
  // one scratch block: cand | off | vic | fits | victim
  const size_t words = (size_t)n_cand + (n_cand + 1) + nv + n_cand + (nv + 3) / 4;
  if (words > ctx->pre_words) {
    if ((rc = dalloc(ctx, &ctx->d_pre, words))) return rc;
    ctx->pre_words = words;
  }
  int32_t* d_cand = ctx->d_pre;
  int32_t* d_off = d_cand + n_cand;
  int32_t* d_vic = d_off + n_cand + 1;
  int32_t* d_fits = d_vic + nv;
  uint8_t* d_victim = reinterpret_cast<uint8_t*>(d_fits + n_cand);
  HIPC(ctx, hipSetDevice(ctx->device));
  HIPC(ctx, hipMemcpyAsync(d_cand, cand_node, sizeof(int32_t) * n_cand, hipMemcpyHostToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(d_off, vic_off, sizeof(int32_t) * (n_cand + 1), hipMemcpyHostToDevice, ctx->stream));
  if (nv) HIPC(ctx, hipMemcpyAsync(d_vic, vic_pod, sizeof(int32_t) * nv, hipMemcpyHostToDevice, ctx->stream));
  // a preemptor whose PodTopologySpread / InterPodAffinity filter reads the
  // node's pods: the topology dry run (ksched_preempt.h), else Fit only
  const bool topo = needs_topo(ctx, ctx->prof, pod, 1);
  int32_t topo_ok = 1;
  if (topo) {
    // refuse on the host what the dry run cannot hold, before any launch
    if ((rc = check_supported(ctx, ctx->prof, pod, 1))) return rc;
    if (preempt_n_ma(ctx, p) > kPreMaxMAnti)
      return fail(ctx, KSG_E_UNSUPPORTED, "preemption: more than " + std::to_string(kPreMaxMAnti) +
                                              " existing anti-affinity templates match the preemptor");
    if (!ctx->d_pretopo) {
      if ((rc = dalloc(ctx, &ctx->d_pretopo, 1))) return rc;
      if ((rc = dalloc(ctx, &ctx->d_preprof, 1))) return rc;
    }
    HIPC(ctx, hipMemcpyAsync(ctx->d_preprof, &ctx->prof, sizeof(ksg_profile), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(ksg_preempt_prepass<1024>, dim3(1), dim3(1024), 0, ctx->stream, ctx->c, ctx->st, ctx->d_pods,
                       ctx->d_prog, ctx->d_preprof, pod, ctx->d_pretopo);
    hipLaunchKernelGGL(ksg_preempt_topo, dim3((n_cand + 255) / 256), dim3(256), 0, ctx->stream, ctx->c, ctx->st,
                       ctx->d_pods, ctx->d_prog, ctx->d_preprof, pod, ctx->d_pretopo, d_cand, n_cand, d_off, d_vic,
                       d_fits, d_victim, ports_on ? 1 : 0);
    HIPC(ctx, hipMemcpyAsync(&topo_ok, &ctx->d_pretopo->ok, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  } else {
    hipLaunchKernelGGL(ksg_preempt_kernel, dim3((n_cand + 255) / 256), dim3(256), 0, ctx->stream, ctx->c, ctx->st,
                       ctx->d_pods, ctx->d_prog, pod, ctx->prof.fit_ignored_res, fit_on ? 1 : 0, ports_on ? 1 : 0,
                       d_cand, n_cand, d_off, d_vic, d_fits, d_victim);
  }
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipMemcpyAsync(fits, d_fits, sizeof(int32_t) * n_cand, hipMemcpyDeviceToHost, ctx->stream));
  if (nv) HIPC(ctx, hipMemcpyAsync(victim, d_victim, nv, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  if (!topo_ok) return fail(ctx, KSG_E_UNSUPPORTED, "preemption: topology terms exceed the dry run's limits");
  return KSG_OK;
}

int ksg_run_replicas(ksg_ctx* ctx, const ksg_profile* profiles, int32_t n_replicas, int32_t first, int32_t count,
                     int32_t* placements, ksg_replica_summary* summaries) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!profiles || n_replicas <= 0 || first < 0 || count < 0 || first + count > ctx->n_pods || !placements)
    return fail(ctx, KSG_E_INVALID, "replica arguments");
  if ((rc = check_blobs(ctx, first, count))) return rc;
  if ((rc = flush_stage(ctx))) return rc;
  if ((rc = flush_commit(ctx))) return rc;
  for (int r = 0; r < n_replicas; r++)
    if ((rc = check_supported(ctx, profiles[r], first, count))) return rc;
  ctx->pct_valid = false;   // (replica state is a copy; conservatively rebuilt)
  HIPC(ctx, hipSetDevice(ctx->device));
  const DevCluster& c = ctx->c;
  const size_t N = c.N, R = c.R, S = std::max(c.S, 1), NT = std::max(c.n_tmpl, 1);
  const size_t RR = n_replicas;
  QueueArgs a = base_args(ctx);
  a.first = first;
  a.count = count;
  a.do_commit = 1;
  Tmp tmp;
  DevState& s = a.st;
  s.stride_req = R * N; s.stride_nz = 2 * N; s.stride_pc = N; s.stride_cnt = S * N; s.stride_tab = ctx->tab_words;
  s.stride_tt = NT; s.stride_part = N; s.stride_sraw = 4 * N;
  bool sweep = sweep_eligible(ctx, profiles, (int)RR, first, count) && count > 0;
  if (ctx->force_path == 1) sweep = false;
  // narrow records when every range check passes (host: pods and profiles,
  // ksg_narrow_init: nodes), else the int64 columns
  int4* nstat = nullptr;
  int4* nmut = nullptr;
  const double2* nrcp = nullptr;
  NarrowBounds nb{};
  if (sweep && narrow_candidate(ctx, profiles, (int)RR, first, count, sweep_mode(profiles, (int)RR), &nb)) {
    unsigned* d_bad;
    TA(tmp, &nstat, sizeof(int4) * N);
    TA(tmp, &nmut, sizeof(int4) * RR * N);
    TA(tmp, &d_bad, 16);
    HIPC(ctx, hipMemsetAsync(d_bad, 0, 16, ctx->stream));
    hipLaunchKernelGGL(ksg_narrow_init, dim3((unsigned)((N + 255) / 256), (unsigned)std::min<size_t>(RR, 64)), dim3(256),
                       0, ctx->stream, ctx->c, ctx->st, nstat, nmut, (int)RR, nb, d_bad);
    HIPC(ctx, hipGetLastError());
    unsigned bad = 0;
    HIPC(ctx, hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(ctx, hipStreamSynchronize(ctx->stream));
    if (bad) nstat = nullptr, nmut = nullptr;
    else nrcp = ctx->c.rcp64;
  }
  ctx->last_narrow = nstat != nullptr;
  // the sweep reads and writes only the Fit columns; the queue kernels also
  // keep the PodTopologySpread / InterPodAffinity tables and per-node scratch
  if (!nstat) {
    TA(tmp, &s.requested, 8 * RR * s.stride_req);
    TA(tmp, &s.nonzero, 8 * RR * s.stride_nz);
    TA(tmp, &s.pod_count, 4 * RR * s.stride_pc);
  }
  s.ports = nullptr;   // replicas never share the context's UsedPorts
  if (!sweep && range_has_ports(ctx, first, count)) {
    s.stride_ports = (size_t)ctx->c.PW * N;
    TA(tmp, &s.ports, 4 * RR * s.stride_ports);
  }
  if (!sweep) {
    TA(tmp, &s.cnt, 4 * RR * s.stride_cnt);
    TA(tmp, &s.tab, 4 * RR * s.stride_tab);
    TA(tmp, &s.tmpl_total, 4 * RR * s.stride_tt);
    TA(tmp, &s.partial, 8 * RR * s.stride_part);
    TA(tmp, &s.sraw, 8 * RR * s.stride_sraw);
  }
  ksg_profile* d_prof;
  int32_t* d_pl;
  int64_t* d_sums;
  TA(tmp, &d_prof, sizeof(ksg_profile) * RR);
  TA(tmp, &d_pl, sizeof(int32_t) * RR * count);
  TA(tmp, &d_sums, sizeof(int64_t) * 2 * RR);
  // every replica starts from the ctx's current state
  auto bcast = [&](auto* src, auto* dst, size_t len, size_t stride) {
    using T = std::remove_pointer_t<decltype(dst)>;
    const unsigned bx = (unsigned)std::min<size_t>((len + 255) / 256, 64);
    hipLaunchKernelGGL(ksg_broadcast<T>, dim3(std::max(bx, 1u), (unsigned)RR), dim3(256), 0, ctx->stream,
                       (const T*)src, dst, len, stride);
  };
  if (!nstat) {
    bcast(ctx->st.requested, s.requested, s.stride_req, s.stride_req);
    bcast(ctx->st.nonzero, s.nonzero, s.stride_nz, s.stride_nz);
    bcast(ctx->st.pod_count, s.pod_count, s.stride_pc, s.stride_pc);
  }
  if (!sweep) {
    bcast(ctx->st.cnt, s.cnt, s.stride_cnt, s.stride_cnt);
    bcast(ctx->st.tab, s.tab, s.stride_tab, s.stride_tab);
    bcast(ctx->st.tmpl_total, s.tmpl_total, s.stride_tt, s.stride_tt);
  }
  if (s.ports) bcast(ctx->st.ports, s.ports, s.stride_ports, s.stride_ports);
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipMemcpyAsync(d_prof, profiles, sizeof(ksg_profile) * RR, hipMemcpyHostToDevice, ctx->stream));
  a.profiles = d_prof;
  a.placements = d_pl;
  a.results = nullptr;
  if (sweep) {
    if ((rc = run_sweep(ctx, a, profiles, d_prof, (int)RR, first, count, d_pl, tmp, nstat, nrcp, nmut, nb.nx))) return rc;
    ctx->last_path = 3;
  } else {
    const int block = N >= 8192 ? 512 : 256;
    bool topo = false;
    for (size_t r = 0; r < RR && !topo; r++) topo = needs_topo(ctx, profiles[r], first, count);
    if ((rc = launch_queue(ctx, a, (int)RR, block, topo))) return rc;
    ctx->last_path = 1;
  }
  HIPC(ctx, hipMemcpyAsync(placements, d_pl, sizeof(int32_t) * RR * count, hipMemcpyDeviceToHost, ctx->stream));
  std::vector<int64_t> sums(2 * RR);
  if (summaries && nmut) {
    hipLaunchKernelGGL(ksg_narrow_sums, dim3((unsigned)RR), dim3(256), 0, ctx->stream, (const int4*)nmut, (int)N,
                       nb.nx >= 0 ? 0xffffffu : 0xffffffffu, d_sums);
    HIPC(ctx, hipGetLastError());
    HIPC(ctx, hipMemcpyAsync(sums.data(), d_sums, sizeof(int64_t) * 2 * RR, hipMemcpyDeviceToHost, ctx->stream));
  } else if (summaries) {
    hipLaunchKernelGGL(ksg_replica_sums, dim3((unsigned)RR), dim3(256), 0, ctx->stream, (const int64_t*)s.requested,
                       s.stride_req, (int)N, d_sums);
    HIPC(ctx, hipGetLastError());
    HIPC(ctx, hipMemcpyAsync(sums.data(), d_sums, sizeof(int64_t) * 2 * RR, hipMemcpyDeviceToHost, ctx->stream));
  }
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIPC(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->last_ms = ms;
  if ((rc = tcollect(ctx))) return rc;
  if (ctx->last_path == 3 && ctx->sweep_timeout) {
    unsigned to = 0;
    HIPC(ctx, hipMemcpy(&to, ctx->sweep_timeout, sizeof(to), hipMemcpyDeviceToHost));
    ctx->sweep_timeout = nullptr;
    if (to) {
      if (ctx->coop_launch) return fail(ctx, KSG_E_DEVICE, "replica sweep: group barrier timed out (cooperative launch)");
      // not every workgroup was resident: every replica starts from the
      // context's state, which the sweep does not change, so the same call
      // runs once more with cooperative launches (from now on)
      ctx->coop_launch = true;
      ctx->recoveries++;
      return ksg_run_replicas(ctx, profiles, n_replicas, first, count, placements, summaries);
    }
  }
  if (summaries) {
    for (size_t r = 0; r < RR; r++) {
      ksg_replica_summary& sm = summaries[r];
      sm = ksg_replica_summary{};
      uint64_t h = 14695981039346656037ull;  // FNV-1a 64 offset basis
      for (int k = 0; k < count; k++) {
        const int32_t v = placements[r * count + k];
        (v >= 0 ? sm.scheduled : sm.unschedulable) += 1;
        for (int b = 0; b < 4; b++) { h ^= (uint8_t)(((uint32_t)v) >> (8 * b)); h *= 1099511628211ull; }
      }
      sm.placement_hash = h;
      sm.cpu_requested = sums[2 * r];
      sm.mem_requested = sums[2 * r + 1];
    }
  }
  return KSG_OK;
}

int ksg_read_state(ksg_ctx* ctx, ksg_node_state* out) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !out) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "no nodes loaded");
  HIPC(ctx, hipSetDevice(ctx->device));
  int rc;
  if ((rc = flush_commit(ctx))) return rc;
  const size_t N = ctx->c.N, R = ctx->c.R;
  if (out->requested) HIPC(ctx, hipMemcpyAsync(out->requested, ctx->st.requested, 8 * R * N, hipMemcpyDeviceToHost, ctx->stream));
  if (out->nonzero) HIPC(ctx, hipMemcpyAsync(out->nonzero, ctx->st.nonzero, 16 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (out->pod_count) HIPC(ctx, hipMemcpyAsync(out->pod_count, ctx->st.pod_count, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

int ksg_reset_state(ksg_ctx* ctx) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx) return KSG_E_INVALID;
  if (!ctx->have_nodes) return fail(ctx, KSG_E_STATE, "no nodes loaded");
  HIPC(ctx, hipSetDevice(ctx->device));
  ctx->pc_node = -1;   // a deferred assume is reset with the rest
  ctx->pct_valid = false;
  const size_t N = ctx->c.N, R = ctx->c.R;
  HIPC(ctx, hipMemcpyAsync(ctx->st.requested, ctx->d_req0, 8 * R * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(ctx->st.nonzero, ctx->d_nz0, 16 * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemcpyAsync(ctx->st.pod_count, ctx->d_pc0, 4 * N, hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.cnt, 0, 4 * std::max(ctx->c.S, 1) * N, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.tab, 0, 4 * ctx->tab_words, ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.tmpl_total, 0, 4 * std::max(ctx->c.n_tmpl, 1), ctx->stream));
  HIPC(ctx, hipMemsetAsync(ctx->st.ports, 0, 4 * (size_t)ctx->c.PW * N, ctx->stream));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  return KSG_OK;
}

#ifdef KSG_STAMPS
// Diagnostic build only: cycle sums per phase-2 segment since load.
int ksg_debug_stamps(ksg_ctx* ctx, unsigned long long* out8) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first   // 16 segment sums
  if (!ctx || !out8 || !ctx->d_stamps) return KSG_E_STATE;
  HIPC(ctx, hipMemcpy(out8, ctx->d_stamps, 128, hipMemcpyDeviceToHost));
  return KSG_OK;
}
// eval_node_src's 16 segment sums (g_eval_stamp)
int ksg_debug_eval_stamps(ksg_ctx* ctx, unsigned long long* out16) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !out16) return KSG_E_INVALID;
  HIPC(ctx, hipSetDevice(ctx->device));
  HIPC(ctx, hipStreamSynchronize(ctx->stream));
  HIPC(ctx, hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_eval_stamp), 128, 0, hipMemcpyDeviceToHost));
  return KSG_OK;
}
#endif

int ksg_set_timing(ksg_ctx* ctx, int on) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx) return KSG_E_INVALID;
  ctx->timing = on != 0;
  treset(ctx);
  return KSG_OK;
}

int ksg_kernel_stats(ksg_ctx* ctx, ksg_kernel_stat* out, int32_t max, int32_t* n) {
  if (int rc_ = srv_stop(ctx)) return rc_;   // the persistent per-cycle server leaves first
  if (!ctx || !n || (max > 0 && !out)) return KSG_E_INVALID;
  int k = 0;
  for (int i = 0; i < KSG_NKERNELS; i++) {
    if (!ctx->kstat_calls[i]) continue;
    if (k < max) {
      ksg_kernel_stat& st = out[k];
      st = ksg_kernel_stat{};
      std::snprintf(st.name, sizeof(st.name), "%s", kKernelNames[i]);
      st.kind = i;
      st.calls = ctx->kstat_calls[i];
      st.total_ms = ctx->kstat_ms[i];
      st.units = ctx->kstat_units[i];
    }
    k++;
  }
  *n = k;
  return KSG_OK;
}

int ksg_topo_window_stats(ksg_ctx* ctx, int64_t* windows, int64_t* pods, int64_t* cut) {
  if (!ctx || !windows || !pods || !cut) return KSG_E_INVALID;
  const bool w = ctx->last_window;
  *windows = w ? (int64_t)ctx->win_stats[0] : 0;
  *pods = w ? (int64_t)ctx->win_stats[1] : 0;
  *cut = w ? (int64_t)ctx->win_stats[2] : 0;
  return KSG_OK;
}

int ksg_recoveries(ksg_ctx* ctx, int32_t* n) {
  if (!ctx || !n) return KSG_E_INVALID;
  *n = ctx->recoveries;
  return KSG_OK;
}

int ksg_last_run_info(ksg_ctx* ctx, int32_t* path, int32_t* flags) {
  if (!ctx || !path || !flags) return KSG_E_INVALID;
  *path = ctx->last_path;
  *flags = (ctx->last_narrow ? KSG_RUN_NARROW_SWEEP : 0) | (ctx->last_n32 ? KSG_RUN_SLOT32 : 0) |
           (ctx->last_spec ? KSG_RUN_SPEC : 0) |
           (ctx->last_mw ? KSG_RUN_WIDE_MEM : 0) | (ctx->last_window ? KSG_RUN_TOPO_WINDOW : 0);
  return KSG_OK;
}

int ksg_last_kernel_ms(ksg_ctx* ctx, double* ms) {
  if (!ctx || !ms) return KSG_E_INVALID;
  *ms = ctx->last_ms;
  return KSG_OK;
}

}  // extern "C"
