#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_r3y.sh $1 && bash scripts/gpu_r3z.sh $1
