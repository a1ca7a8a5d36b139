#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/slot2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"; grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k['name'],k['calls'],round(k['avg_ms'],4)) for k in d['roofline']['kernels']]"
timeout -k 10 120 python -u profiles/stamps.py 20000 > $O/stamps.log 2>&1; echo "stamps rc=$?"; cat $O/stamps.log | tail -6
