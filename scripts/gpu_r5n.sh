#!/bin/bash
# annotation sidecars: host vs device serialiser throughput and digests
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/annot_bench.py 2000 256 > $O/annot.json 2> $O/annot.err || { echo "annot failed"; tail -20 $O/annot.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5n/annot.json"))
for k, v in d.items():
    dv = v.get("device_serialiser") or {}
    print(k, "host", round(v["pods_per_s"]), v["digest_xxh3"], "capture-only", round(v["capture_only_pods_per_s"]),
          "| device", round(dv.get("pods_per_s", 0)), dv.get("digest_xxh3"), dv.get("bytes_equal_host"), dv.get("error"))
PY
