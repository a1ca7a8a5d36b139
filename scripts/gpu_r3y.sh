#!/bin/bash
# Round-3: per-cycle C driver, topo-coop stamps, configs[2] + configs[4] benches, headline bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u scripts/percycle.py 5000 500 2000 > $O/percycle.json 2> $O/percycle.err; rc=$?
echo "percycle rc=$rc"; cat $O/percycle.json
[ $rc -eq 0 ] || { tail -20 $O/percycle.err; exit 1; }
timeout -k 10 300 python -u profiles/stamps_topo.py 3000 > $O/stamps_topo.txt 2> $O/stamps_topo.err; rc=$?
echo "stamps rc=$rc"; cat $O/stamps_topo.txt
[ $rc -eq 0 ] || { tail -20 $O/stamps_topo.err; exit 1; }
timeout -k 10 300 python -u scripts/bench_configs.py --config 5 --no-cpu-baseline > $O/config5.json 2> $O/config5.err; rc=$?
echo "config5 rc=$rc"; python -c "import json;d=json.load(open('$O/config5.json'));print(d['pods_per_s'], [(k['name'],round(k['avg_ms'],4),round(k['frac'],3)) for k in d['roofline']['kernels']])"
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --sweep-replicas 0 --annotate-pods 0 --default-pods 0 --no-cpu-baseline --cycle-pods 0 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 1200 $O/bench.json | head -c 600; echo
exit $rc
