#!/bin/bash
# Per-cycle kernel variants: default (plain stores + one release), system-scope
# stores (KSG_CYCLE_SYS=1), 4-byte rows (KSG_CYCLE_ES=4): stamps + C-driver timing.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_eval.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "base" "KSG_CYCLE_SYS=1" "KSG_CYCLE_ES=4"; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env $e timeout -k 10 200 python3 -u profiles/stamps_cycle.py 5000 1000 > $O/stamps_$v.txt 2>&1 || { echo "stamps $v failed"; tail -5 $O/stamps_$v.txt; exit 1; }
  env $e timeout -k 10 200 python3 -u scripts/percycle.py 5000 500 2000 > $O/pc_$v.json 2> $O/pc_$v.err || { echo "percycle $v failed"; tail -5 $O/pc_$v.err; exit 1; }
  echo "== $v"; cat $O/stamps_$v.txt | head -9; python3 -c "import json,sys; d=json.load(open('$O/pc_$v.json')); print(round(d['us_per_cycle_mean'],1), d['breakdown_us_mean'])"
done
