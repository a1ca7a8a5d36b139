#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_snapshot_c.py tests/test_gpu_snapshot.py tests/test_gpu_parity.py -k "eval or snapshot or c_boundary or kat or readme" -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 300 python -u scripts/percycle.py 5000 500 2000 > $O/percycle$i.json 2> $O/percycle$i.err; rc=$?
echo "percycle rc=$rc"; cat $O/percycle$i.json
[ $rc -eq 0 ] || exit 1
done
exit 0
