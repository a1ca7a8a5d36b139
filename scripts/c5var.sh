# config-5 sweep variants (group size); measurement script, see DESIGN.md §4.4
set -o pipefail
for v in "KSG_SWEEP_S=8" "KSG_SWEEP_S=4" "KSG_SWEEP_S=16"; do
  echo "== $v" >> gpurun_out/c5var.log
  env $v timeout -k 10 200 python -u scripts/bench_configs.py --config 5 --pods 256 --reps 2 --no-cpu-baseline >> gpurun_out/c5var.log 2>&1 || exit 1
done
