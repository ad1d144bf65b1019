#!/bin/bash
# Tile-length sweep of the per-rank shard of an 8-GPU strong-scaling run (1,250 cells of
# configs[3]) beside the 10k-cell step on the same box: step and pass time per tile length,
# and the one-launch step (pert_enum_step) at the planner's length.
# usage: tools/shard_lt_sweep.sh TAG [cells] [lt ...]
set -o pipefail
TAG=${1:-run}; shift || true
CELLS=${1:-1250}; shift || true
LTS=${*:-"30 34 36 38 40 42 46 54"}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_lt_sweep.log
: > $OUT
row() {   # label, bench args
  local label=$1; shift
  timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${TAG}_lt.tmp 2>&1 || { tail -5 gpurun_out/${TAG}_lt.tmp; exit 1; }
  python -c "
import json, sys
r = json.loads(open('gpurun_out/${TAG}_lt.tmp').read().strip().splitlines()[-1])
rf = r['roofline']; pc = rf.get('pattern_ceiling', {})
print('$label', 'cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'], 4),
      'pass_ms', round(rf['kernel_ms'], 4), 'ceiling_ms', round(pc.get('ms', 0), 4), 'frac_ceiling', round(pc.get('kernel_frac_of_ceiling', 0), 3))
" | tee -a $OUT
}
row c4_auto
row shard_auto --cells $CELLS
row shard_auto_fused --cells $CELLS --fused
for lt in $LTS; do
  row shard_lt$lt --cells $CELLS --bins-per-tile $lt
done
row c4_auto_again
