#!/bin/bash
# Step-1 tile length (per-cell partial volume vs pass occupancy) and the shard's tile length,
# interleaved on one box.
set -o pipefail
TAG=${1:-r04n}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_sweep.log
: > $OUT
row() {
  local label=$1; shift
  timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  python -c "
import json
r = json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); rf = r['roofline']
print('$label', r['config']['fit'], 'cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'], 4), 'pass_ms', round(rf['kernel_ms'], 4))
" | tee -a $OUT
}
for rep in 1 2; do
  for lt in 0 150 210 300; do row s1 --fit step1 --bins-per-tile $lt || exit 1; done
  for lt in 0 54; do row shard --cells 1250 --bins-per-tile $lt || exit 1; done
done
