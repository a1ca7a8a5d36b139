#!/bin/bash
# The batched placement path on one MI355X: parity tests (pytest -k expression),
# the stamped spec-walk breakdown, then the phase-2 modes side by side.
# Usage: bash scripts/gpu_spec.sh <out-subdir> [modes] [pytest -k expression]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-spec}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_batch_variants.py tests/test_gpu_parity.py -k "${3:-spec}" -x -v --timeout 300 --timeout-method thread > $O/spec_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 $O/spec_tests.log
[ $rc -eq 0 ] || exit 1
if [ -f kube-scheduler-simulator_amd/libksched_stamps.so ]; then
  KSG_BATCH_MODE=spec timeout -k 10 200 python -u profiles/stamps.py 20000 > $O/stamps_spec.txt 2>&1; rc=$?
  echo "stamps rc=$rc"; cat $O/stamps_spec.txt
  [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 400 python -u scripts/compare_modes.py --modes ${2:-window,spec} > $O/modes.log 2>&1; rc=$?
echo "modes rc=$rc"; cat $O/modes.log | cut -c1-400
exit $rc
