#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_json.py  > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -15 $O/tests.txt
timeout -k 10 300 python3 -u scripts/annot_dev.py 2000 256 > $O/dev.txt 2>&1 || { echo "dev failed"; tail -20 $O/dev.txt; exit 1; }
cut -c1-1500 $O/dev.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 -u scripts/annot_dev.py 2000 256 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
for f in $(find $O/prof -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 "$f" | head -14; done
