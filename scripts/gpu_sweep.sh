#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-sweep}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_parity.py -k "sweep or replicas" -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/tests.log | tail -25
[ $rc -eq 0 ] || exit 1
shift || true
bash scripts/gpu_configs.sh ${O#gpurun_out/}/cfg "$@"
