#!/bin/bash
# Non-headline configs on one GPU (scripts/bench_configs.py), one JSON line each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-configs}
mkdir -p $O
shift || true
i=0
for a in "$@"; do
  i=$((i+1))
  echo "== $a"
  timeout -k 10 300 python -u scripts/bench_configs.py $a > $O/c$i.json 2> $O/c$i.log || { echo "failed: $a"; tail -5 $O/c$i.log; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/c$i.json')); r=d['roofline']; print(d['workload'], '| dev %.1f ms pods/s %.0f evals/s %.3g | %s %.1f GB/s frac %.3f' % (d['device_ms'], d['pods_per_s'], d['node_evals_per_s'], r['kernel'], r['achieved'], r['frac']))"
done
