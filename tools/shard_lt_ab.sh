#!/bin/bash
# Interleaved A/B of tile lengths for the per-rank shard of an 8-GPU strong-scaling run (1,250
# cells of configs[3]), three rounds on one box, with the 10k step between rounds (the
# projection's numerator from the same box).
# usage: tools/shard_lt_ab.sh TAG [lt ...]
set -o pipefail
TAG=${1:-run}; shift || true
LTS=${*:-"40 42 54"}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_lt_ab.log
: > $OUT
row() {
  local label=$1; shift
  timeout -k 10 120 python bench.py --steps 60 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${TAG}_ab.tmp 2>&1 || { tail -5 gpurun_out/${TAG}_ab.tmp; exit 1; }
  python -c "
import json
r = json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); rf = r['roofline']
print('$label', 'cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'], 4),
      'pass_ms', round(rf['kernel_ms'], 4), 'ceiling_ms', round(rf.get('pattern_ceiling', {}).get('ms', 0), 4))
" | tee -a $OUT
}
for rep in 1 2 3; do
  row c4 || exit 1
  for lt in $LTS; do
    row shard_lt$lt --cells 1250 --bins-per-tile $lt || exit 1
  done
done
