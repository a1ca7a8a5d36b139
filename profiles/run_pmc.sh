#!/bin/bash
# Profiles on one MI355X (run from the repo root on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of the headline bench (default profile
#      at 5,000 x 50,000) and of configs[1] (bench.py --workload configs1)
#   2. PMC passes FETCH_SIZE and WRITE_SIZE (separate runs) of the same two
#   3. the same three for the config-4 replica sweep (scripts/bench_configs.py)
#   4. TOPO=1: configs[2]'s topology kernel (kernel trace, FETCH / WRITE, SQ mix)
#   5. CYCLE=1: the per-cycle path (scripts/percycle.py)
# SKIP_BENCH / SKIP_SWEEP drop parts 1-2 / 3.
# Summaries are folded by profiles/pmc_summary.py into profiles/rNN/.
set -uo pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
# a PMC pass prints nothing until it ends: keep a heartbeat under gpurun_out/
( while sleep 45; do date >> "$OUT/heartbeat.txt"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --configs1-pods 0 --sweep-replicas 0 --annotate-pods 0 --cycle-pods 0 --kubelet-pods 0 --topo-cycle-pods 0 --topo-annotate-pods 0"
B1="$B --workload configs1"
S="python3 scripts/bench_configs.py --config 4 --replicas 1024 --pods 256 --reps 1 --no-cpu-baseline"
SP="$S --no-timing"
run() {  # name, rocprof args..., -- command
  local name=$1; shift
  # every profiled process must exit 0: native handles are closed by an
  # atexit hook (native.track), and a crash at exit is a failure, not noise
  KSG_EXIT_MAPS="$OUT/$name.maps" timeout -k 10 240 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$OUT/$name.log"; exit 1; }
}
if [ -z "${SKIP_BENCH:-}" ]; then
run bench_kt --kernel-trace --stats --output-format csv -d "$OUT/bench_kt" -o run -- $B
# counter passes serialise kernels: the window pipeline on one stream (same
# arithmetic), else each walk would wait out its poll for the other stream
export KSG_PIPE_OVERLAP=0
run bench_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/bench_fetch" -o run -- $B
run bench_write --pmc WRITE_SIZE --output-format csv -d "$OUT/bench_write" -o run -- $B
unset KSG_PIPE_OVERLAP
run c1_kt --kernel-trace --stats --output-format csv -d "$OUT/c1_kt" -o run -- $B1
export KSG_PIPE_OVERLAP=0
run c1_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/c1_fetch" -o run -- $B1
run c1_write --pmc WRITE_SIZE --output-format csv -d "$OUT/c1_write" -o run -- $B1
unset KSG_PIPE_OVERLAP
fi
if [ -z "${SKIP_SWEEP:-}" ]; then
run sweep_kt --kernel-trace --stats --output-format csv -d "$OUT/sweep_kt" -o run -- $S
run sweep_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/sweep_fetch" -o run -- $SP
run sweep_write --pmc WRITE_SIZE --output-format csv -d "$OUT/sweep_write" -o run -- $SP
fi
# 4. configs[2] (TOPO=1): the chip-wide topology kernel, 3,000 pods at
#    15,000 nodes: kernel trace, FETCH_SIZE, WRITE_SIZE and the SQ issue / wait mix
if [ -n "${TOPO:-}" ]; then
T="python3 scripts/bench_configs.py --config 3 --pods 3000 --reps 1 --no-cpu-baseline"
run topo_kt --kernel-trace --stats --output-format csv -d "$OUT/topo_kt" -o run -- $T
run topo_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/topo_fetch" -o run -- $T --no-timing
run topo_write --pmc WRITE_SIZE --output-format csv -d "$OUT/topo_write" -o run -- $T --no-timing
run topo_sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/topo_sq" -o run -- $T --no-timing
fi
# 4b. configs[4] (CONFIG5=1): 64 replicas x 100,000 nodes, first 500 pods
if [ -n "${CONFIG5:-}" ]; then
F="python3 scripts/bench_configs.py --config 5 --replicas 64 --pods 500 --reps 1 --no-cpu-baseline"
run c5_kt --kernel-trace --stats --output-format csv -d "$OUT/c5_kt" -o run -- $F
run c5_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/c5_fetch" -o run -- $F --no-timing
run c5_write --pmc WRITE_SIZE --output-format csv -d "$OUT/c5_write" -o run -- $F --no-timing
fi
# 5. the per-cycle path (CYCLE=1): 2,000 cycles at 5,000 nodes through the C driver
if [ -n "${CYCLE:-}" ]; then
C="python3 scripts/percycle.py 5000 500 2000"
run cycle_kt --kernel-trace --stats --output-format csv -d "$OUT/cycle_kt" -o run -- $C
export KSG_PIPE_OVERLAP=0   # the driver's closing queue check runs the batched path (see part 2)
run cycle_fetch --pmc FETCH_SIZE --output-format csv -d "$OUT/cycle_fetch" -o run -- $C
run cycle_write --pmc WRITE_SIZE --output-format csv -d "$OUT/cycle_write" -o run -- $C
unset KSG_PIPE_OVERLAP
fi
find "$OUT" -name "*.csv" | sort
