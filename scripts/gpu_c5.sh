#!/bin/bash
# configs[4] (64 replicas x 100,000 nodes): its GPU tests, the bench line and
# the sweep's kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-c5}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
F="python3 scripts/bench_configs.py --config 5 --replicas 64 --pods 500 --reps 1 --no-cpu-baseline"
timeout -k 10 300 $F > "$O/c5.json" 2> "$O/c5.err" || { echo "bench failed"; tail -5 "$O/c5.err"; exit 1; }
tail -c 400 "$O/c5.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- $F > "$O/kt.log" 2>&1 || { echo "trace failed"; tail -5 "$O/kt.log"; exit 1; }
f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/c5_kernel_stats.csv"; head -4 "$O/c5_kernel_stats.csv"
find "$O/kt" -name "*kernel_trace.csv" -delete
