#!/bin/bash
# configs[2]: segment stamps of the topology kernel, the full 150,000-pod queue timed
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u profiles/stamps_topo.py 3000 > $O/stamps_topo.txt 2>&1 || { echo "stamps failed"; tail -20 $O/stamps_topo.txt; exit 1; }
cat $O/stamps_topo.txt
timeout -k 10 400 python3 -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 --no-cpu-baseline --save-placements $O/c3_150k_placements.npy > $O/c3_full.json 2> $O/c3_full.err || { echo "c3 failed"; tail -20 $O/c3_full.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3_full.json')); print({k: d[k] for k in ('value','unit','ms_per_step') if k in d}, d.get('roofline'))"
