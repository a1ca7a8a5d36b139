#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_snapshot.py tests/test_volumes.py tests/test_snapshot_c.py -m gpu > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -25 $O/tests.txt
timeout -k 10 900 python3 -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 --pmc profiles/r5/pmc_config3.json > $O/config3_full.json 2> $O/config3_full.err || { echo "config3 failed"; tail -20 $O/config3_full.err; exit 1; }
cut -c1-1200 $O/config3_full.json
