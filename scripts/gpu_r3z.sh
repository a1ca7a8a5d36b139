#!/bin/bash
# Round-3: per-cycle kernel trace; configs[2] group-size sweep.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cycle -o cyc -- python3 scripts/percycle.py 5000 200 1000 > $O/percycle_prof.log 2>&1; rc=$?
echo "percycle prof rc=$rc"; tail -3 $O/percycle_prof.log
[ $rc -eq 0 ] || exit 1
for g in 30 15; do
  KSG_COOP_GMAX=$g timeout -k 10 300 python -u scripts/bench_configs.py --config 3 --pods 3000 --no-cpu-baseline > $O/config3_g$g.json 2> $O/config3_g$g.err; rc=$?
  echo "config3 gmax=$g rc=$rc"; python -c "import json;d=json.load(open('$O/config3_g$g.json'));print(d['pods_per_s'], d['device_ms'])"
  [ $rc -eq 0 ] || exit 1
done
exit 0
