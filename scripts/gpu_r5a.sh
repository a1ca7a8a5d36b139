#!/bin/bash
# Round 5, first box: smoke, targeted GPU tests, the new headline bench, and
# the exit-crash check under rocprofv3 (with the atexit close; then, last, the
# old behaviour with /proc/self/maps recorded to map the crash).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_eval.py tests/test_snapshot_c.py tests/test_snapshot_native.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
echo "bench ok"
KSG_EXIT_MAPS=$O/pc_close.maps timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pc_close -o run -- python3 -u scripts/percycle.py 5000 500 2000 > $O/pc_close.log 2>&1
echo "percycle under rocprofv3, handles closed at exit: rc=$?"
KSG_NO_EXIT_CLOSE=1 KSG_EXIT_MAPS=$O/pc_open.maps timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pc_open -o run -- python3 -u scripts/percycle.py 5000 500 2000 > $O/pc_open.log 2>&1
echo "percycle under rocprofv3, handles left open: rc=$?"
