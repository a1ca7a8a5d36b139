#!/bin/bash
# One GPU session: parity tests, topset opt-in tests, bench in both phase-2 modes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r1s2
mkdir -p $O
run() { local name=$1; shift; echo "== $name"; "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.log; return $rc; }
run gpu_tests timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run topset_tests timeout -k 10 300 python -u -m pytest tests -m topset -x -q --timeout 120 --timeout-method thread; rc=$?
[ $rc -eq 0 ] || exit 0
run bench_scan timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 || exit 1
KSG_BATCH_MODE=topset run bench_topset timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
exit 0
