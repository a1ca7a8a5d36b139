#!/bin/bash
# The speculate-and-verify walk on one MI355X: its parity tests, then the
# phase-2 modes side by side.  Usage: bash scripts/gpu_spec.sh <out-subdir> [modes]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-spec}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_variants.py -k "spec" -x -v --timeout 300 --timeout-method thread > $O/spec_tests.log 2>&1; rc=$?
echo "spec tests rc=$rc"; tail -15 $O/spec_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/compare_modes.py --modes ${2:-window,spec} > $O/modes.log 2>&1; rc=$?
echo "modes rc=$rc"; cat $O/modes.log | cut -c1-400
exit $rc
