#!/bin/bash
# The per-cycle topology tables: the per-cycle / eval / snapshot / preemption
# / C-boundary GPU tests, then the per-cycle legs of the bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pctables}
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_snapshot.py tests/test_preemption.py tests/test_snapshot_c.py tests/test_gpu_topo_coop.py -m gpu > "$O/tests.txt" 2>&1 || { echo "tests failed"; tail -40 "$O/tests.txt"; exit 1; }
tail -3 "$O/tests.txt"
timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --configs1-pods 0 --sweep-replicas 0 --annotate-pods 0 --kubelet-pods 0 --topo-annotate-pods 0 > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
for k in ("per_cycle", "per_cycle_server", "per_cycle_configs2"):
    v = d.get(k)
    print(k, v and (round(v["us_per_cycle_mean"], 1), round(v["us_per_cycle_p50"], 1),
                    {a: round(b, 1) for a, b in v["breakdown_us_mean"].items()}, v.get("placements_equal_run_queue")))
PY
if [ -f kube-scheduler-simulator_amd/libksched_stamps.so ]; then
  timeout -k 10 300 python3 -u profiles/stamps_topo.py 1600 eval > "$O/stamps_eval.txt" 2>&1 || { echo "stamps failed"; tail -5 "$O/stamps_eval.txt"; exit 1; }
  cat "$O/stamps_eval.txt"
fi
