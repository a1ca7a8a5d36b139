#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5w
mkdir -p $O
export TMPDIR=/tmp
KSG_DUMP_MAPS=$O/maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 -u scripts/annot_dev.py 1024 64 c3 > $O/prof.log 2>&1
echo "rc=$?"
grep -A25 "SIGSEGV" $O/prof.log | head -30
