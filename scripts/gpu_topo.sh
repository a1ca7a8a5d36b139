#!/bin/bash
# Round-3: topology path (configs[2]): parity tests, stamps, the full queue.
O=gpurun_out/${1:-r3t0}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_topo_coop.py tests/test_preemption.py tests/test_gpu_eval.py tests/test_gpu_parity.py} > $O/topo_tests.log 2>&1; rc=$?
echo "topo tests rc=$rc"; tail -3 $O/topo_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/topo_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u profiles/stamps_topo.py 3000 > $O/stamps_topo.txt 2> $O/stamps_topo.err; rc=$?
echo "stamps rc=$rc"; cat $O/stamps_topo.txt
[ $rc -eq 0 ] || { tail -20 $O/stamps_topo.err; exit 1; }
timeout -k 10 300 python3 -u scripts/bench_configs.py --config 3 --pods 150000 --reps 1 ${2:+--no-cpu-baseline} > $O/config3.json 2> $O/config3.err; rc=$?
echo "config3 rc=$rc"; python3 -c "import json;d=json.load(open('$O/config3.json'));print(d['pods_per_s'], d['device_ms'], d['scheduled'])"
