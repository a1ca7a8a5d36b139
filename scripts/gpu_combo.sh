#!/bin/bash
# spec-walk parity + modes, then the round's PMC passes and configs[2] full queue.
# Usage: bash scripts/gpu_combo.sh <out-subdir>
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-combo}
bash scripts/gpu_spec.sh $O spec "spec or c2 or readme" || exit 1
bash scripts/gpu_pmc_r3.sh $O
