#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-coop}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_topo_coop.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/stamps_topo.py 3000 > $O/stamps.log 2>&1; echo "stamps rc=$?"; cat $O/stamps.log
bash scripts/gpu_configs.sh ${O#gpurun_out/}/cfg "--config 3 --pods 3000"
