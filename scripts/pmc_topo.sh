#!/bin/bash
# SQ counters of the chip-wide topology kernel (issue vs wait), two passes; run from the repo root on the GPU box.
set -uo pipefail
OUT=${1:-gpurun_out/pmc_topo}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 scripts/bench_configs.py --config 3 --pods 640 --reps 1 --no-timing --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/a" -o run -- $B > "$OUT/a.log" 2>&1 || { tail -5 "$OUT/a.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM --output-format csv -d "$OUT/b" -o run -- $B > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    avg = {c: v / max(1, n[(k, c)]) for c, v in d.items()}
    print(k, {c: round(v, 1) for c, v in sorted(avg.items())})
    w = avg.get("SQ_WAVES")
    if w and "topo_coop" in k:
        pods = 64
        print("  per pod and wave:", {c: round(avg[c] / w / pods, 1) for c in avg if c.startswith("SQ_INSTS")},
              {c: round(4 * avg[c] / w / pods, 1) for c in avg if "CYCLES" in c or "WAIT" in c or "ACTIVE" in c})
PY
