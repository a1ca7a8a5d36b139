#!/bin/bash
# Round-3 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) of the bench and
# the config-4 sweep, then configs[2] on the whole 150,000-pod queue.
# Usage: bash scripts/gpu_pmc_r3.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
mkdir -p $O
bash profiles/run_pmc.sh $O/pmc || exit 1
( while sleep 45; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 > $O/config3_full.json 2> $O/config3_full.err; rc=$?
echo "config3 rc=$rc"; tail -2 $O/config3_full.err; cut -c1-400 $O/config3_full.json
exit $rc
