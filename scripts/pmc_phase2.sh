#!/bin/bash
# SQ counters of the phase-2 slot kernel (issue vs wait), one pass; run from the repo root on the GPU box.
set -uo pipefail
OUT=${1:-gpurun_out/pmc_p2}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --pods 5120 --sweep-replicas 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/a" -o run -- $B > "$OUT/a.log" 2>&1 || { tail -5 "$OUT/a.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM --output-format csv -d "$OUT/b" -o run -- $B > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / max(1, n[(k, c)]), 1) for c, v in sorted(d.items())})
PY
