#!/bin/bash
# SQ instruction and wait mix of the config-2 bench kernels on one MI355X (run
# from the repo root on the GPU box); each counter pass is its own run under a
# hard time limit.  Summarised by profiles/sq_summary.py.
set -uo pipefail
OUT=${1:-gpurun_out/sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
export KSG_PIPE_OVERLAP=0   # counter passes serialise kernels (see run_pmc.sh)
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --sweep-replicas 0 --annotate-pods 0 --default-pods 0 --cycle-pods 0"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $B > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit 1; }
}
pass sq_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pass sq_b SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS
pass sq_c SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SENDMSG SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_SALU SQ_WAVES
