#!/bin/bash
# Per-cycle A/B on one box: one launch per cycle vs the persistent server,
# interleaved (configs[1], 5,000 nodes, 2,000 timed cycles each).
# Usage (on the box): bash scripts/gpu_pc_ab.sh <out-subdir> [reps]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pcab}
mkdir -p "$O"
for r in $(seq 1 "${2:-2}"); do
  for m in launch server; do
    timeout -k 10 240 python3 -u scripts/percycle.py 5000 500 2000 c2 $m > "$O/${m}_$r.json" 2> "$O/${m}_$r.err" || { echo "$m $r failed"; tail -5 "$O/${m}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/${m}_$r.json')); print('$m', $r, round(d['us_per_cycle_mean'],2), round(d['us_per_cycle_p50'],2), {k: round(v,2) for k,v in d['breakdown_us_mean'].items()}, d['placements_equal_run_queue'])"
  done
done
