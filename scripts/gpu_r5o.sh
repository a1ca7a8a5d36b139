#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/annot_dev.py 2000 256 > $O/dev.txt 2>&1 || { echo "failed"; tail -20 $O/dev.txt; exit 1; }
cat $O/dev.txt | cut -c1-1500
