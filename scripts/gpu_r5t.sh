#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --sweep-replicas 0 --cycle-pods 0 --topo-cycle-pods 0 --kubelet-pods 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open("gpurun_out/r5t/bench.json").read().strip().splitlines()[-1])
for k in ("annotations","annotations_configs2"):
    print(k, json.dumps(d[k].get("device_serialiser")))
PY
