#!/bin/bash
# Phase-2 modes side by side on one MI355X (plain library), then the stamped breakdown.
# Usage: bash scripts/gpu_modes.sh <out-subdir> <modes> [pods]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-modes}
mkdir -p $O
timeout -k 10 400 python -u scripts/compare_modes.py --modes ${2:-window,spec} --pods ${3:-50000} > $O/modes.log 2>&1; rc=$?
echo "modes rc=$rc"; cat $O/modes.log | cut -c1-400
[ $rc -eq 0 ] || exit 1
KSG_BATCH_MODE=spec timeout -k 10 200 python -u profiles/stamps.py 20000 > $O/stamps_spec.txt 2>&1; rc=$?
echo "stamps rc=$rc"; cat $O/stamps_spec.txt | tail -12
exit $rc
