#!/bin/bash
# Per-cycle legs with the statuses delta form (default) and the dense form
# (KSG_DRIVER_DENSE=1), interleaved on one box, configs[1] and configs[2].
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-st_ab}
mkdir -p "$O"
for rep in 1 2; do
  for c in "5000 500 2000 c2" "15000 300 400 c3"; do
    for d in 0 1; do
      set -- $c
      if [ $d = 1 ]; then export KSG_DRIVER_DENSE=1; else unset KSG_DRIVER_DENSE; fi
      timeout -k 10 300 python3 -u scripts/percycle.py $1 $2 $3 $4 > "$O/pc_${4}_${d}_${rep}.json" 2>> "$O/err.txt" || { echo "percycle failed"; tail -20 "$O/err.txt"; exit 1; }
      python3 - "$O/pc_${4}_${d}_${rep}.json" "$4 dense=$d" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["us_per_cycle_mean"], 1), round(d["us_per_cycle_p50"], 1),
      {a: round(b, 1) for a, b in d["breakdown_us_mean"].items()}, d["placements_equal_run_queue"])
PY
    done
  done
done
