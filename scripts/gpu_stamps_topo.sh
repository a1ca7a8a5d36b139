#!/bin/bash
# Stamped breakdown (KSG_STAMPS build) of the chip-wide topology kernel:
# the configs[2] queue path and the per-cycle form (one pod per launch), the
# latter with and without the per-cycle domain tables.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-stamps_topo}
mkdir -p "$O"
timeout -k 10 300 python3 -u profiles/stamps_topo.py 3000 > "$O/queue.txt" 2>&1 || { echo queue failed; tail -5 "$O/queue.txt"; exit 1; }
timeout -k 10 300 python3 -u profiles/stamps_topo.py 1600 eval > "$O/eval.txt" 2>&1 || { echo eval failed; tail -5 "$O/eval.txt"; exit 1; }
KSG_PC_TABLES=0 timeout -k 10 300 python3 -u profiles/stamps_topo.py 1600 eval > "$O/eval_notables.txt" 2>&1 || { echo eval0 failed; tail -5 "$O/eval_notables.txt"; exit 1; }
cat "$O/queue.txt" "$O/eval.txt" "$O/eval_notables.txt"
