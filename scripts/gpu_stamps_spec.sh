#!/bin/bash
# Stamped segments of the speculate-and-verify walk (the KSG_STAMPS build):
# configs[1] and the headline's default profile, 20,000 pods each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-stamps_spec}
mkdir -p $O
KSG_BATCH_MODE=spec timeout -k 10 300 python3 -u profiles/stamps.py 20000 > $O/c1.txt 2>&1 || { echo c1 failed; tail -5 $O/c1.txt; exit 1; }
KSG_BATCH_MODE=spec timeout -k 10 300 python3 -u profiles/stamps.py 20000 default > $O/def.txt 2>&1 || { echo def failed; tail -5 $O/def.txt; exit 1; }
cat $O/c1.txt $O/def.txt
