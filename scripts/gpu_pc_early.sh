#!/bin/bash
# The per-cycle topology tests, then configs[2] per cycle with the phase-2
# rows written after barrier 2 (KSG_CYCLE_EARLY=1, default) and in 3c (0),
# interleaved on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pc_early}
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_snapshot.py tests/test_snapshot_c.py tests/test_gpu_topo_coop.py -m gpu > "$O/tests.txt" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for rep in 1 2 3; do
  for e in 1 0; do
    KSG_CYCLE_EARLY=$e timeout -k 10 300 python3 -u scripts/percycle.py 15000 300 400 c3 > "$O/pc_${e}_$rep.json" 2>> "$O/err.txt" || { echo "percycle $e failed"; tail -20 "$O/err.txt"; exit 1; }
    python3 - "$O/pc_${e}_$rep.json" "early=$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["us_per_cycle_mean"], 1), round(d["us_per_cycle_p50"], 1),
      {a: round(b, 1) for a, b in d["breakdown_us_mean"].items()}, d["placements_equal_run_queue"])
PY
  done
done
