#!/bin/bash
# Round 5: the rebuilt per-cycle kernel (one-wave workgroups, argument-carried
# pod, prefetched node columns): parity tests, per-cycle timing, stamps and a
# kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_eval.py tests/test_snapshot_c.py tests/test_snapshot_native.py tests/test_gpu_ingest.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -u scripts/percycle.py 5000 500 2000 > $O/pc1.json 2> $O/pc1.err || { echo "percycle failed"; tail -20 $O/pc1.err; exit 1; }
timeout -k 10 200 python3 -u scripts/percycle.py 5000 500 2000 > $O/pc2.json 2> $O/pc2.err || { echo "percycle 2 failed"; tail -20 $O/pc2.err; exit 1; }
cat $O/pc1.json $O/pc2.json
timeout -k 10 200 python3 -u profiles/stamps_cycle.py 5000 1000 > $O/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cyc_kt -o run -- python3 -u scripts/percycle.py 5000 500 2000 > $O/cyc_kt.log 2>&1 || { echo "rocprof failed rc=$?"; tail -20 $O/cyc_kt.log; exit 1; }
find $O/cyc_kt -name "*kernel_stats.csv" | xargs head -4
