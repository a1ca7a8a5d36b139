#!/bin/bash
# Round-3 closing evidence: suite, smoke, bench, kernel trace, then PMC passes.
# Usage: bash scripts/gpu_close_r3.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-close}
bash scripts/gpu_round_end.sh $O || exit 1
export TMPDIR=/tmp
bash profiles/run_pmc.sh gpurun_out/$O/pmc
