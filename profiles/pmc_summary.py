"""Fold rocprofv3 outputs of profiles/run_pmc.sh into per-kernel summaries.

  python profiles/pmc_summary.py <run_pmc out dir> <dest dir>

Writes <dest>/{bench,c1,sweep,topo,cycle,c5}_kernel_stats.csv (the --stats
summaries, copied), <dest>/pmc_{default,config2,config4,config3,per_cycle,config5}.json and,
where an SQ pass ran, <dest>/sq_<config>.json (average counter values per
dispatch).  pmc_*.json: per kernel, dispatches, average
FETCH_SIZE and WRITE_SIZE per dispatch (KB as rocprofv3 reports them) and HBM
bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (x 1024): the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of
wide coalesced reads; WRITE_SIZE exact).  The sweep/bench kernels read 8-byte
words per lane, a width the guide leaves uncalibrated, so the raw counters are
kept beside the corrected figure.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def kernel_key(name: str) -> str:
    """The ksg_kernel_stats name of a rocprofv3 kernel name: template
    arguments dropped, except that the narrow replica-sweep instances
    (ksg_sweep<..., NARROW = true>, the sixth argument) are ksg_sweep_narrow."""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0].strip()
    base = name.split("<")[0].strip()
    ns = base[:base.rindex("::") + 2] if "::" in base else ""   # (ksk::)
    if base == ns + "ksg_sweep" and "<" in name:
        args = [a.strip() for a in name[name.index("<") + 1:name.rindex(">")].split(",")]
        if len(args) >= 6 and args[5] == "true":
            return ns + "ksg_sweep_narrow"
    if base == ns + "ksg_topo_coop" and "<" in name:   # CAP = 3: the speculative topology queue's window rows
        args = [a.strip() for a in name[name.index("<") + 1:name.rindex(">")].split(",")]
        if len(args) >= 3 and args[2] == "3":
            return ns + "ksg_topo_coop_window"
    return base


def counters(path):
    """{kernel: [values per dispatch]} from a counter_collection.csv."""
    out = defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                name = kernel_key(name)
                out[name].append(float(row["Counter_Value"]))
    return out


def counters_by_name(path):
    """{kernel: {counter: average per dispatch}} from a multi-counter pass."""
    acc, n = defaultdict(lambda: defaultdict(float)), defaultdict(int)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                n[(k, row["Counter_Name"])] += 1
    return {k: {c: v / n[(k, c)] for c, v in sorted(d.items())} for k, d in acc.items()}


def main():
    src, dest = sys.argv[1], sys.argv[2]
    os.makedirs(dest, exist_ok=True)
    for tag, cfg in (("bench", "default"), ("c1", "config2"), ("sweep", "config4"), ("topo", "config3"), ("cycle", "per_cycle"),
                     ("c5", "config5")):
        if not glob.glob(os.path.join(src, f"{tag}_*")):
            continue
        sq = counters_by_name(os.path.join(src, f"{tag}_sq"))
        if sq:
            json.dump(sq, open(os.path.join(dest, f"sq_{cfg}.json"), "w"), indent=1)
        for f in glob.glob(os.path.join(src, f"{tag}_kt", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dest, f"{tag}_kernel_stats.csv"))
        fetch, write = counters(os.path.join(src, f"{tag}_fetch")), counters(os.path.join(src, f"{tag}_write"))
        res = {}
        for k in sorted(set(fetch) | set(write)):
            fv, wv = fetch.get(k, []), write.get(k, [])
            fa = sum(fv) / len(fv) if fv else None
            wa = sum(wv) / len(wv) if wv else None
            res[k] = {"dispatches": max(len(fv), len(wv)), "fetch_size_kb": fa, "write_size_kb": wa,
                      "hbm_bytes_per_dispatch": None if fa is None or wa is None else (2 * fa + wa) * 1024}
        json.dump(res, open(os.path.join(dest, f"pmc_{cfg}.json"), "w"), indent=1)
        print(cfg, json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
