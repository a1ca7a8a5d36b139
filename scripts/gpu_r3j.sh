#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_snapshot_c.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u scripts/percycle.py 5000 500 2000 > $O/percycle.json 2> $O/percycle.err; rc=$?
echo "percycle rc=$rc"; cat $O/percycle.json
[ $rc -eq 0 ] || { tail -20 $O/percycle.err; exit 1; }
timeout -k 10 300 python -u profiles/stamps_topo.py 3000 > $O/stamps_topo.txt 2> $O/stamps_topo.err; rc=$?
echo "stamps rc=$rc"; cat $O/stamps_topo.txt
exit $rc
