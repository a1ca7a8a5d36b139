#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u scripts/percycle.py 5000 500 2000 > $O/percycle.json 2> $O/percycle.err; rc=$?
echo "percycle rc=$rc"; cat $O/percycle.json
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/prof_cycle -o cyc -- python3 scripts/percycle.py 5000 200 600 > $O/percycle_prof.log 2>&1; rc=$?
echo "percycle prof rc=$rc"
[ $rc -eq 0 ] || exit 1
bash scripts/pmc_topo.sh $O/pmc_topo > $O/pmc_topo.log 2>&1; rc=$?
echo "pmc topo rc=$rc"; tail -6 $O/pmc_topo.log
exit $rc
