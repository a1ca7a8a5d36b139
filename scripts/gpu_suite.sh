#!/bin/bash
# GPU session: the full -m gpu suite, then smoke (driver's round-end order).
# Usage (on the box, from the repo root): bash scripts/gpu_suite.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
exit $rc
