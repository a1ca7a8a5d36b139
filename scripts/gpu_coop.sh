#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-coop}
mkdir -p $O
shift || true
timeout -k 10 500 python -u -m pytest tests/test_gpu_topo_coop.py tests/test_gpu_parity.py -k "coop or placement_queue" -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert|Timeout" $O/tests.log | tail -30
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_configs.sh ${O#gpurun_out/}/cfg "$@"
