#!/bin/bash
# The configs[2] per-cycle path: the per-cycle GPU tests, then a same-box A/B
# of the staged in-place read (KSG_TOPO_STAGE), the one-pod completion
# (KSG_CYCLE_LAST), the per-cycle tables (KSG_PC_TABLES) and the by-value
# commit (KSG_COMMIT_ARGS), interleaved, then
# the GPU timeline of the default form under rocprofv3.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pc_ab}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_eval.py tests/test_gpu_snapshot.py tests/test_preemption.py tests/test_snapshot_c.py tests/test_gpu_topo_coop.py} -m gpu > "$O/tests.txt" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for rep in 1 2; do
  for v in "1 1 1 1" "0 1 1 1" "1 1 1 0" "1 1 0 1"; do
    set -- $v
    KSG_TOPO_STAGE=$1 KSG_CYCLE_LAST=$2 KSG_PC_TABLES=$3 KSG_COMMIT_ARGS=${4:-1} timeout -k 10 300 python3 -u scripts/percycle.py 15000 300 400 c3 > "$O/pc_$1$2$3${4:-1}_$rep.json" 2>> "$O/err.txt" || { echo "percycle $v failed"; tail -20 "$O/err.txt"; exit 1; }
    python3 - "$O/pc_$1$2$3${4:-1}_$rep.json" "stage=$1 last=$2 tables=$3 args=${4:-1}" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["us_per_cycle_mean"], 1), round(d["us_per_cycle_p50"], 1),
      {a: round(b, 1) for a, b in d["breakdown_us_mean"].items()}, d["placements_equal_run_queue"])
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 -u scripts/percycle.py 15000 300 400 c3 > "$O/prof.txt" 2>&1 || { echo "prof failed"; tail -20 "$O/prof.txt"; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
grep -i "topo\|commit\|copy" "$f" | cut -c1-160
