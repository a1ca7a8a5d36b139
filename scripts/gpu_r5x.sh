#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_json.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python3 -u scripts/annot_dev.py 4000 256 > $O/dev_c1.txt 2>&1 || { echo "dev failed"; tail -20 $O/dev_c1.txt; exit 1; }
grep rep $O/dev_c1.txt
timeout -k 10 300 python3 -u scripts/annot_dev.py 1024 64 c3 > $O/dev_c3.txt 2>&1 || { echo "dev c3 failed"; tail -20 $O/dev_c3.txt; exit 1; }
grep rep $O/dev_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 -u scripts/annot_dev.py 2000 256 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
for f in $(find $O/prof -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
