#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b2
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --configs1-pods 0 --sweep-replicas 0 --annotate-pods 0 --kubelet-pods 0 --topo-annotate-pods 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r5b2/bench.json").read().strip().splitlines()[-1])
for k in ("per_cycle","per_cycle_server","per_cycle_configs2"):
    v=d.get(k); print(k, v and (round(v["us_per_cycle_mean"],1), round(v["us_per_cycle_p50"],1), {a: round(b,1) for a,b in v["breakdown_us_mean"].items()}, v.get("full_reloads"), v.get("placements_equal_run_queue")))
print("headline", d["value"], d["roofline"].get("traffic"))
PY
