#!/bin/bash
# Per-cycle path after a row-width change: its GPU tests, the per-cycle legs
# (server and launch, interleaved), and the server's FETCH / WRITE passes.
# Usage (on the box): bash scripts/gpu_pc_rows.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pcrows}
mkdir -p "$O"
export TMPDIR=/tmp
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_eval.py \
  tests/test_snapshot_c.py tests/test_gpu_recovery.py > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.log"; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 "$O/tests.log"
[ -n "${SKIP_AB:-}" ] || bash scripts/gpu_pc_ab.sh "${1:-pcrows}/ab" 2 || exit 1
C="python3 scripts/percycle.py 5000 500 2000"
mkdir -p "$O/pmc"
export KSG_PIPE_OVERLAP=0   # counter passes serialise kernels (run_pmc.sh part 5)
for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
  n=${pass%%:*}; c=${pass##*:}
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$O/pmc/cycle_$n" -o run -- $C > "$O/pmc/cycle_$n.log" 2>&1 || { echo "$c failed"; tail -20 "$O/pmc/cycle_$n.log"; exit 1; }
  echo "$c ok"
done
python3 profiles/pmc_summary.py "$O/pmc" "$O/summary" > "$O/pmc.log" 2>&1 || tail -5 "$O/pmc.log"
cat "$O/summary/pmc_per_cycle.json" | head -30
find "$O/pmc" -name "*.csv" -size +2M -delete
