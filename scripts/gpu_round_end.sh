#!/bin/bash
# Closing GPU session: the -m gpu suite, smoke, the default bench line, and
# rocprofv3 kernel stats of the bench.  Usage: bash scripts/gpu_round_end.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-end}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -2 $O/bench.err; grep '^{' $O/bench.json | cut -c1-400
[ $rc -eq 0 ] || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_kt -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --sweep-replicas 0 --annotate-pods 0 --default-pods 0 --cycle-pods 0 > $O/bench_kt.log 2>&1; rc=$?
echo "rocprof rc=$rc"; head -8 $O/bench_kt/run_kernel_stats.csv
exit $rc
