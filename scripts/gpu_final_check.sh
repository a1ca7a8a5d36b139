#!/bin/bash
# Round-3 last check on the committed tree: smoke and the default bench line.
O=gpurun_out/${1:-r3fin}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench.json
