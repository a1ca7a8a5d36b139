#!/bin/bash
# Full GPU check: every -m gpu test, smoke(), default bench, stamps breakdown.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['cpu_baseline']); [print(k['name'],k['calls'],round(k['avg_ms'],4)) for k in d['roofline']['kernels']]"
timeout -k 10 120 python -u profiles/stamps.py 20000 > $O/stamps.log 2>&1; echo "stamps rc=$?"; tail -6 $O/stamps.log
