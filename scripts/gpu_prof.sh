#!/bin/bash
# Stamps breakdown of phase 2 + rocprofv3 kernel trace of the default bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/prof1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/stamps.py 20000 > $O/stamps.log 2>&1; echo "stamps rc=$?"; cat $O/stamps.log | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/bench_prof.log 2>&1; echo "prof rc=$?"
find $O/kt -name "*kernel_stats.csv" | xargs cat
