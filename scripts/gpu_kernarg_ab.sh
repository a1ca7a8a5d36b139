#!/bin/bash
# Headline A/B: kernel arguments in host memory (HIP default) vs device memory
# (HIP_FORCE_DEV_KERNARG=1), interleaved on one box, headline + configs[1].
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-kernarg}
mkdir -p "$O"
B="python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --sweep-replicas 0 --annotate-pods 0 --cycle-pods 0 --kubelet-pods 0 --topo-cycle-pods 0 --topo-queue-pods 0 --topo-annotate-pods 0"
for r in 1 2; do
  for m in 0 1; do
    HIP_FORCE_DEV_KERNARG=$m timeout -k 10 300 $B > "$O/k${m}_$r.json" 2> "$O/k${m}_$r.err" || { echo "run $m $r failed"; tail -5 "$O/k${m}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/k${m}_$r.json').read().strip().splitlines()[-1]); print('kernarg_dev=$m', $r, round(d['value']), round(d['ms_per_step'],2), round(d['configs1']['pods_per_s']))"
  done
done
