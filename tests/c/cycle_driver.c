/* Per-cycle timing driver (bench.py per_cycle sidecar): the calls the Go shim
 * makes per scheduling cycle, in C, timed call by call with CLOCK_MONOTONIC,
 * so the measured cost is the C ABI's alone (no Python / ctypes in the loop):
 *
 *   ksg_snapshot_add_pod -> ksg_snapshot_sync -> ksg_eval_view (the rows
 *   in library memory) -> ksg_snapshot_statuses_kept (the snapshot's arrays,
 *   kept across cycles) -> ksg_snapshot_assume
 *
 * hint_ahead > 0: cycle i first announces pod i + hint_ahead
 * (ksg_snapshot_hint_pod, timed with add_pod), as the Go shim's pod informer
 * does for a pod created while the queue runs.
 *
 * Bench infrastructure, not product: links libksched.so only. */
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include "ksched.h"
#include "ksched_snapshot.h"

static int64_t now_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000000000ll + t.tv_nsec;
}

/* views[n]: the pods in queue order.  Cycles i >= warm record their five
 * phase times (ns) in phase_ns[(i - warm) * 5 ..].  placed[n]: selected node
 * or -1.  *appended / *reloads: syncs of the timed cycles that appended /
 * re-encoded.  Returns 0 or the failing call's code (negative), with *where
 * naming the phase. */
int cycle_run(ksg_snapshot* s, ksg_ctx* ctx, const ksg_pod_view* views, int32_t n, int32_t warm,
              ksg_eval_rows* rows, int32_t n_nodes, int32_t* placed, int64_t* phase_ns, int32_t* appended,
              int32_t* reloads, int32_t* where, int32_t hint_ahead) {
  int32_t* code = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nodes);
  int32_t* msg = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nodes);
  const int64_t cap_bytes = 1 << 16;
  char* buf = (char*)malloc((size_t)cap_bytes);
  int rc = 0;
  const int dense = getenv("KSG_DRIVER_DENSE") != NULL;   /* measurement: the dense statuses form */
  *appended = *reloads = 0;
  for (int32_t i = 0; i < n && rc == 0; i++) {
    int32_t idx = -1, ap = 0, n_msgs = 0;
    int64_t len = 0;
    ksg_result r;
    const int64_t t0 = now_ns();
    if (hint_ahead > 0 && i + hint_ahead < n && (rc = ksg_snapshot_hint_pod(s, &views[i + hint_ahead]))) {
      *where = 0;
      break;
    }
    if ((rc = ksg_snapshot_add_pod(s, &views[i], &idx))) { *where = 0; break; }
    const int64_t t1 = now_ns();
    if ((rc = ksg_snapshot_sync(s, ctx, &ap))) { *where = 1; break; }
    const int64_t t2 = now_ns();
    if ((rc = ksg_eval_view(ctx, idx, &r, rows))) { *where = 2; break; }
    const int64_t t3 = now_ns();
    const int32_t *kcode = NULL, *kmsg = NULL;
    if ((rc = dense ? ksg_snapshot_statuses(s, idx, rows->fstatus, n_nodes, code, msg, buf, cap_bytes, &n_msgs, &len)
                    : ksg_snapshot_statuses_kept(s, idx, rows->fstatus, n_nodes, &kcode, &kmsg, buf, cap_bytes,
                                                 &n_msgs, &len))) {
      *where = 3;
      break;
    }
    const int64_t t4 = now_ns();
    if (r.selected >= 0 && (rc = ksg_snapshot_assume(s, ctx, idx, r.selected))) { *where = 4; break; }
    const int64_t t5 = now_ns();
    placed[i] = r.selected;
    if (i >= warm) {
      int64_t* ph = phase_ns + (size_t)(i - warm) * 5;
      ph[0] = t1 - t0;
      ph[1] = t2 - t1;
      ph[2] = t3 - t2;
      ph[3] = t4 - t3;
      ph[4] = t5 - t4;
      *appended += ap != 0;
      *reloads += ap == 0;
    }
  }
  free(code);
  free(msg);
  free(buf);
  return rc;
}
