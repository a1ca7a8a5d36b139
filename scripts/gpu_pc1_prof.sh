#!/bin/bash
# configs[1] per-cycle path under rocprofv3: the GPU timeline of a cycle.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pc1_prof}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/percycle.py 5000 500 2000 c2 > "$O/pc.json" 2>&1 || { echo "percycle failed"; tail -20 "$O/pc.json"; exit 1; }
tail -c 600 "$O/pc.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/prof" -o run -- python3 -u scripts/percycle.py 5000 500 2000 c2 > "$O/prof.txt" 2>&1 || { echo "prof failed"; tail -20 "$O/prof.txt"; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
cut -c1-150 "$f" | head -12
