#!/bin/bash
# Which bench leg leaves the process faulting at exit under rocprofv3: one
# traced bench per leg (the headline plus that leg), stopping at the first
# non-zero exit.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-exit_bisect}
mkdir -p "$O"
export TMPDIR=/tmp
Z="--no-cpu-baseline --steps 1 --warmup 1 --configs1-pods 0 --sweep-replicas 0 --annotate-pods 0 --cycle-pods 0 --kubelet-pods 0 --topo-cycle-pods 0 --topo-annotate-pods 0"
leg() {
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- python3 -u bench.py $Z "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
leg cycle --cycle-pods 2000 && leg topo_cycle --topo-cycle-pods 400 && leg annotate --annotate-pods 2000 --topo-annotate-pods 256 && leg sweep_c1 --sweep-replicas 1024 --configs1-pods 50000 && leg kubelet --kubelet-pods 50000
