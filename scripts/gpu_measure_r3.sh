#!/bin/bash
# Round-3 measurement session on one MI355X (repo root on the box):
#   1. the default bench line (driver contract, CPU baseline, every sidecar)
#   2. rocprofv3 kernel trace + FETCH/WRITE PMC passes of the bench and of the config-4 sweep
#   3. configs[2] on the whole 150,000-pod queue with its CPU baseline
# Usage: bash scripts/gpu_measure_r3.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-measure}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -2 $O/bench.err; cut -c1-300 $O/bench.json
[ $rc -eq 0 ] || exit 1
bash profiles/run_pmc.sh $O/pmc || exit 1
timeout -k 10 300 python -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 > $O/config3_full.json 2> $O/config3_full.err; rc=$?
echo "config3 rc=$rc"; tail -2 $O/config3_full.err; cut -c1-300 $O/config3_full.json
exit $rc
