#!/bin/bash
# Volume plugins, RequestedToCapacityRatio replica sweeps, and the main parity files on the GPU
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_volumes.py tests/test_gpu_sweep.py tests/test_gpu_parity.py tests/test_gpu_eval.py tests/test_gpu_ingest.py \
  tests/test_snapshot_c.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
