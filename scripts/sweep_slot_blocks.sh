#!/bin/bash
# GPU: batch-variant parity, the config-2 bench at each slot block size, and the
# stamped phase-2 breakdown (diagnostic build).  Run from the repo root.
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch_variants.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/variants.log 2>&1
for b in ${BLOCKS:-256 128 64}; do
  KSG_SLOT_BLOCK=$b timeout -k 10 200 python bench.py --steps 3 --no-cpu-baseline --sweep-replicas 0 > gpurun_out/bench_b$b.json 2>gpurun_out/bench_b$b.err
done
for b in ${STAMP_BLOCKS:-256}; do
  KSG_SLOT_BLOCK=$b timeout -k 10 200 python profiles/stamps.py 20000 > gpurun_out/stamps_b$b.txt 2>&1
done
