#!/bin/bash
# configs[2] full queue: the speculative topology queue vs ksg_topo_coop pod
# by pod, interleaved on one box.  Usage: bash scripts/gpu_c3_ab.sh <out> [pods]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-c3ab}
mkdir -p "$O"
P=${2:-150000}
for m in 1 0; do
  KSG_TOPO_WINDOW=$m timeout -k 10 400 python3 -u scripts/bench_configs.py --config 3 --pods $P --reps 2 --no-cpu-baseline \
    > "$O/c3_window$m.json" 2> "$O/c3_window$m.err" || { echo "window=$m failed"; tail -5 "$O/c3_window$m.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_window$m.json')); print('window=$m', round(d['pods_per_s']), 'pods/s device', round(d['device_ms'],1), 'ms wall', round(d['wall_ms'],1), d.get('topo_window'), (d['roofline'] or {}).get('kernel'))"
done
