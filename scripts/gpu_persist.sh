#!/bin/bash
# The persistent spec walk: its GPU tests (headline golden, batch variants,
# parity, recovery), then the headline A/B against one launch per batch.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-persist}
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_headline.py \
  tests/test_gpu_batch_variants.py tests/test_gpu_parity.py tests/test_gpu_recovery.py > "$O/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
B="python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --sweep-replicas 0 --annotate-pods 0 --cycle-pods 0 --kubelet-pods 0 --topo-cycle-pods 0 --topo-queue-pods 0 --topo-annotate-pods 0"
for r in 1 2; do
  for m in 0 1; do
    KSG_SPEC_PERSIST=$m timeout -k 10 300 $B > "$O/p${m}_$r.json" 2> "$O/p${m}_$r.err" || { echo "run $m $r failed"; tail -5 "$O/p${m}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/p${m}_$r.json').read().strip().splitlines()[-1]); print('persist=$m', $r, round(d['value']), round(d['ms_per_step'],2), round(d['configs1']['pods_per_s']), d.get('placements_equal_oracle'))"
  done
done
