"""Fold the rocprofv3 SQ passes of profiles/run_sq.sh into per-kernel mixes.

  python profiles/sq_summary.py <run_sq out dir> <dest json>

Per kernel and counter: the average per dispatch.  Per wave: instructions by
class, and the wave's cycles split into issuing (ACTIVE_INST_ANY), parked on
s_waitcnt / s_barrier (WAIT_ANY) and issue stalls (WAIT_INST_ANY); the cycle
counters count quad-cycles (MI355X_MICROARCH.md, rocprofv3 PMC units), so
they are multiplied by 4 here.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import kernel_key  # noqa: E402


def main():
    src, dest = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(src, "sq_*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row.get("Kernel_Name") or "")
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "per_dispatch": avg}
        waves = avg.get("SQ_WAVES") or 0
        if waves:
            per = {}
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"):
                if c in avg:
                    per[c.replace("SQ_INSTS_", "insts_").lower()] = avg[c] / waves
            for c in ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MISC"):
                if c in avg:
                    per[c.replace("SQ_", "cycles_").lower()] = 4 * avg[c] / waves
            d["per_wave"] = per
        out[k] = d
    with open(dest, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, d in out.items():
        if "per_wave" in d:
            print(k, json.dumps({a: round(b) for a, b in d["per_wave"].items()}))


if __name__ == "__main__":
    main()
