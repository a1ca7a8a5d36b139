#!/bin/bash
# The speculative topology queue on the GPU: small cases first, then the
# topology suite, the golden configs[2] queues and the configs[2] throughput.
# Usage (on the box): bash scripts/gpu_topo_win.sh <out-subdir> [full]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-topowin}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_topo_coop.py -x -v --timeout 150 --timeout-method thread \
  -k "c3-4000 or window_sizes or zoo-big-0" > "$O/small.log" 2>&1; rc=$?
echo "small rc=$rc"; tail -4 "$O/small.log"
[ $rc -eq 0 ] || exit 1
[ "${2:-}" = "full" ] || exit 0
timeout -k 10 900 python -u -m pytest tests/test_gpu_topo_coop.py -x -v --timeout 300 --timeout-method thread \
  > "$O/topo.log" 2>&1; rc=$?
echo "topo rc=$rc"; tail -4 "$O/topo.log"
exit $rc
