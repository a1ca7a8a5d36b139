#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/annot_dev.py 1024 64 c3 > $O/dev_c3.txt 2>&1 || { echo "dev failed"; tail -20 $O/dev_c3.txt; exit 1; }
grep rep $O/dev_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 -u scripts/annot_dev.py 1024 64 c3 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
for f in $(find $O/prof -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 "$f" | head -10; done
