#!/bin/bash
# Round-end evidence on one MI355X (repo root on the GPU box): GPU parity of the
# batched variants, the default bench line, then rocprofv3 --kernel-trace --stats
# of the same bench (timed steps only).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_batch_variants.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/final/parity.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/kt -o run -- \
  python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/final/kt.log 2>&1
