#!/bin/bash
# Round-3 session: NodePorts / eval / variant / topology parity, phase-2 modes,
# headline bench, configs[2] bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_node_ports.py tests/test_gpu_eval.py tests/test_gpu_batch_variants.py tests/test_snapshot_c.py tests/test_gpu_topo_coop.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u scripts/bench_configs.py --config 3 --pods 5000 --no-cpu-baseline > $O/config3.json 2> $O/config3.err; rc=$?
echo "config3 rc=$rc"; tail -c 1500 $O/config3.json; echo
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/compare_modes.py --modes window,tcol > $O/modes.log 2>&1; rc=$?
echo "modes rc=$rc"; tail -12 $O/modes.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --sweep-replicas 0 --annotate-pods 0 --default-pods 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 2500 $O/bench.json; echo
exit $rc
