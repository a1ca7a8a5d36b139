#!/bin/bash
# Plain launches of the grid-barrier kernels: the topology and sweep GPU
# tests, then configs[2] (and configs[4]) under rocprofv3 -- every profiled
# process must exit 0 -- their summary, and the full 150,000-pod queue with
# its roofline and the PMC traffic joined in.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pmc_r5z
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topo_coop.py tests/test_gpu_sweep.py tests/test_gpu_json.py -m gpu > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
SKIP_BENCH=1 SKIP_SWEEP=1 TOPO=1 CONFIG5=1 bash profiles/run_pmc.sh $O > $O/run_pmc.txt 2>&1 || { echo "pmc failed"; tail -30 $O/run_pmc.txt; exit 1; }
grep "rc=" $O/run_pmc.txt
python3 profiles/pmc_summary.py $O $O/sum > $O/summary.txt 2>&1 || { echo "summary failed"; tail -20 $O/summary.txt; exit 1; }
ls $O/sum
timeout -k 10 900 python3 -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 --pmc $O/sum/pmc_config3.json > $O/config3_full.json 2> $O/config3_full.err || { echo "config3 failed"; tail -20 $O/config3_full.err; exit 1; }
cut -c1-800 $O/config3_full.json
