#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5d2
mkdir -p $O
B="python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --configs1-pods 0 --sweep-replicas 0 --annotate-pods 0 --kubelet-pods 0 --topo-annotate-pods 0 --cycle-pods 0"
timeout -k 10 400 $B > $O/ll.json 2> $O/ll.err || { echo "ll failed"; tail -20 $O/ll.err; exit 1; }
KSG_COOP_NO_LL=1 timeout -k 10 400 $B > $O/noll.json 2> $O/noll.err || { echo "noll failed"; tail -20 $O/noll.err; exit 1; }
python3 - <<'PY'
import json
for f in ("ll","noll"):
    d=json.loads(open(f"gpurun_out/r5d2/{f}.json").read().strip().splitlines()[-1])
    v=d.get("per_cycle_configs2"); print(f, v and (round(v["us_per_cycle_mean"],1), {a: round(b,1) for a,b in v["breakdown_us_mean"].items()}))
PY
