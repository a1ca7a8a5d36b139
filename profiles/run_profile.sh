#!/bin/bash
# Per-kernel timing of the headline workload under rocprofv3 (run on the GPU box
# from the repo root).  Usage: profiles/run_profile.sh <out-dir> [bench args...]
set -euo pipefail
OUT=${1:-gpurun_out/prof}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --no-cpu-baseline "$@"
