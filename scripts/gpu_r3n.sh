#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
bash scripts/gpu_r3m.sh $1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_topo_coop.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_topo.log 2>&1; rc=$?
echo "topo tests rc=$rc"; tail -2 $O/tests_topo.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests_topo.log | head -20; exit 1; }
timeout -k 10 300 python -u scripts/bench_configs.py --config 3 --pods 5000 --no-cpu-baseline > $O/config3.json 2> $O/config3.err; rc=$?
echo "config3 rc=$rc"; python -c "import json;d=json.load(open('$O/config3.json'));print(d['pods_per_s'], d['device_ms'])"
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u profiles/stamps_topo.py 3000 > $O/stamps_topo.txt 2> $O/stamps_topo.err; rc=$?
echo "stamps rc=$rc"; cat $O/stamps_topo.txt
exit $rc
