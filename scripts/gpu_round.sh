#!/bin/bash
# The round's closing measurement on one MI355X (run from the repo root on the
# GPU box): smoke, the default bench line, the bench under a kernel trace.
# Usage: bash scripts/gpu_round.sh <gpurun_out subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-round}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 "$O/smoke.log"
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"; rc=$?
echo "bench rc=$rc"; tail -c 600 "$O/bench.json"
[ $rc -eq 0 ] || { tail -20 "$O/bench.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bench_kt" -o run -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$O/bench_kt.log" 2>&1; rc=$?
echo "bench kernel trace rc=$rc"
find "$O/bench_kt" -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {}'
exit 0
