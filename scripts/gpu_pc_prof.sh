#!/bin/bash
# Kernel durations of the configs[2] per-cycle path under rocprofv3, per
# completion form (KSG_CYCLE_LAST) and tables (KSG_PC_TABLES).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-pc_prof}
mkdir -p "$O"
export TMPDIR=/tmp
for v in "1 1" "0 1" "1 0"; do
  set -- $v
  KSG_CYCLE_LAST=$1 KSG_PC_TABLES=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$1$2" -o run -- python3 -u scripts/percycle.py 15000 300 400 c3 > "$O/prof$1$2.txt" 2>&1 || { echo "prof $v failed"; tail -20 "$O/prof$1$2.txt"; exit 1; }
  f=$(find "$O/prof$1$2" -name 'run_kernel_stats.csv' | head -1)
  echo "last=$1 tables=$2"; head -1 "$f" | cut -c1-200; grep -i "topo\|commit\|static" "$f" | cut -c1-200
done
