#!/bin/bash
# Round-3 GPU session: selected test files, then optional bench legs.
# usage: gpu_r3.sh OUTDIR "test files..." [bench args...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
TESTS=$2
shift 2
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err; rc=$?
  echo "bench rc=$rc"; tail -c 3000 $O/bench.json; echo
  [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit 1; }
fi
exit 0
