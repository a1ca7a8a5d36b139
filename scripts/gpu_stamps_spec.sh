#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5f2
mkdir -p $O
KSG_BATCH_MODE=spec timeout -k 10 300 python3 -u profiles/stamps.py 20000 > $O/c1.txt 2>&1 || { echo c1 failed; tail -5 $O/c1.txt; exit 1; }
KSG_BATCH_MODE=spec timeout -k 10 300 python3 -u profiles/stamps.py 20000 default > $O/def.txt 2>&1 || { echo def failed; tail -5 $O/def.txt; exit 1; }
cat $O/c1.txt $O/def.txt
