#!/bin/bash
# New plugin args (RequestedToCapacityRatio, PodTopologySpread defaultConstraints) on the GPU
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_eval.py tests/test_gpu_topo_coop.py -k "rtcr or pts or zoo" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
