#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --sweep-replicas 0 --cycle-pods 0 --topo-cycle-pods 0 --kubelet-pods 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r5s/bench.json").read().strip().splitlines()[-1])
for k in ("annotation","annotation_configs2"):
    v=d.get(k) or d.get("sidecars",{}).get(k)
    print(k, json.dumps(v)[:1500] if v else None)
print(list(d.keys()))
PY
