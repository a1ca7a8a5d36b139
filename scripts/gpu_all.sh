#!/bin/bash
# Every -m gpu test, then the given scripts/bench_configs.py runs.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-all}
mkdir -p $O
shift || true
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
if [ -f kube-scheduler-simulator_amd/libksched_stamps.so ]; then
  timeout -k 10 200 python -u profiles/stamps_topo.py 3000 > $O/stamps_topo.log 2>&1; echo "stamps rc=$?"; cat $O/stamps_topo.log
fi
[ $# -gt 0 ] && bash scripts/gpu_configs.sh ${O#gpurun_out/}/cfg "$@"
exit 0
