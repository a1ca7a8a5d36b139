#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/annot_dev.py 4000 256 > $O/dev_one.txt 2>&1 || { echo "dev failed"; tail -20 $O/dev_one.txt; exit 1; }
grep rep $O/dev_one.txt | cut -c1-30
KSG_JSON_SPLIT=1 timeout -k 10 300 python3 -u scripts/annot_dev.py 4000 256 > $O/dev_split.txt 2>&1 || { echo "dev split failed"; tail -20 $O/dev_split.txt; exit 1; }
grep rep $O/dev_split.txt
KSG_JSON_SPLIT=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_json.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
