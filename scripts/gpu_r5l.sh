#!/bin/bash
# per-cycle C driver on configs[2] (15,000 nodes, PTS + IPA): launch and server
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5l
mkdir -p $O
export TMPDIR=/tmp
for m in launch server; do
  timeout -k 10 300 python3 -u scripts/percycle.py 15000 300 1500 c3 $m > $O/pc3_$m.json 2> $O/pc3_$m.err || { echo "percycle $m failed"; tail -5 $O/pc3_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pc3_$m.json')); print('$m', round(d['us_per_cycle_mean'],1), round(d['us_per_cycle_p50'],1), {k: round(v,2) for k,v in d['breakdown_us_mean'].items()}, d.get('eval_path'), d['placements_equal_run_queue'])"
done
