#!/bin/bash
# The device annotation serialiser on one MI355X (run from the repo root on the
# GPU box): its parity tests, per-chunk launch / wait times on configs[1] and
# configs[2] (scripts/annot_dev.py), a kernel + copy trace, and the FETCH_SIZE
# / WRITE_SIZE passes of its kernels (separate runs).  Every step is bounded
# and a failure ends the script.
# Usage: bash scripts/gpu_serialiser.sh <gpurun_out subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-serialiser}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_json.py > "$O/tests.txt" 2>&1 || { echo "tests failed"; tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
timeout -k 10 300 python3 -u scripts/annot_dev.py 4000 256 > "$O/dev_c1.txt" 2>&1 || { echo "configs[1] failed"; tail -20 "$O/dev_c1.txt"; exit 1; }
grep rep "$O/dev_c1.txt" | cut -c1-40
timeout -k 10 300 python3 -u scripts/annot_dev.py 1024 64 c3 > "$O/dev_c3.txt" 2>&1 || { echo "configs[2] failed"; tail -20 "$O/dev_c3.txt"; exit 1; }
grep rep "$O/dev_c3.txt" | cut -c1-40
D="python3 -u scripts/annot_dev.py 1024 256"
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/kt" -o run -- $D > "$O/kt.log" 2>&1 || { echo "trace failed"; tail -5 "$O/kt.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- $D > "$O/fetch.log" 2>&1 || { echo "fetch failed"; tail -5 "$O/fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- $D > "$O/write.log" 2>&1 || { echo "write failed"; tail -5 "$O/write.log"; exit 1; }
for f in $(find "$O/kt" -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
