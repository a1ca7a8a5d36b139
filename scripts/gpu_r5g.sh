#!/bin/bash
# Per-cycle: launch kernel with system-scope stores (default now) and the
# relayed persistent server: parity, stamps, C-driver timing.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_eval.py tests/test_snapshot_c.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "base" "KSG_CYCLE_SERVER=1"; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env $e timeout -k 10 200 python3 -u profiles/stamps_cycle.py 5000 1000 > $O/stamps_$v.txt 2>&1 || { echo "stamps $v failed"; tail -5 $O/stamps_$v.txt; exit 1; }
  echo "== $v"; head -9 $O/stamps_$v.txt
done
for m in launch server; do
  timeout -k 10 200 python3 -u scripts/percycle.py 5000 500 2000 c2 $m > $O/pc_$m.json 2> $O/pc_$m.err || { echo "percycle $m failed"; tail -5 $O/pc_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pc_$m.json')); print('$m', round(d['us_per_cycle_mean'],1), round(d['us_per_cycle_p50'],1), {k: round(v,2) for k,v in d['breakdown_us_mean'].items()}, d['placements_equal_run_queue'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o pc -- python3 -u scripts/percycle.py 5000 500 2000 c2 launch > $O/prof.log 2>&1 || { echo "rocprof failed rc=$?"; tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); grep -i cycle "$f" | cut -c1-200
