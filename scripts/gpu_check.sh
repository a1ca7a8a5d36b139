#!/bin/bash
# Every -m gpu test, smoke(), and the default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit 1
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
  echo "bench rc=$rc"; cat $O/bench.json | head -c 600; echo
fi
exit 0
