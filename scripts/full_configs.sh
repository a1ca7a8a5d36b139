#!/bin/bash
# configs[2..4] at (or near) their BASELINE sizes on one MI355X; run from the repo root on the GPU box.
set -euo pipefail
mkdir -p gpurun_out/full
timeout -k 10 300 python3 -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 > gpurun_out/full/config3.json 2> gpurun_out/full/config3.err
timeout -k 10 300 python3 -u scripts/bench_configs.py --config 4 --pods 50000 --reps 1 > gpurun_out/full/config4.json 2> gpurun_out/full/config4.err
timeout -k 10 400 python3 -u scripts/bench_configs.py --config 5 --pods 2000 --reps 1 > gpurun_out/full/config5.json 2> gpurun_out/full/config5.err
