#!/bin/bash
# The device serialiser's kernels: FETCH_SIZE / WRITE_SIZE passes (separate
# runs) and a kernel trace of scripts/annot_dev.py on configs[1].
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5e2
mkdir -p $O
export TMPDIR=/tmp
D="python3 -u scripts/annot_dev.py 1024 256"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $D > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $D > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $D > $O/write.log 2>&1 || { echo "write failed"; tail -5 $O/write.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/r5e2"
def rows(kind):
    f = glob.glob(f"{O}/{kind}/**/*counter_collection.csv", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []
for kind, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    acc = collections.defaultdict(list)
    for r in rows(kind):
        if "json" in r.get("Kernel_Name", ""):
            acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(kind, k, len(v), "avg KB", round(sum(v) / len(v), 1))
PY
for f in $(find $O/kt -name '*kernel_stats.csv'); do cut -d, -f1-4 "$f" | grep -i json; done
