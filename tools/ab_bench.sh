#!/bin/bash
# Interleaved A/B of the default build against another build of the same ABI (PERT_LIB), three
# rounds on one box: C4 step 2, the 1,250-cell shard and C5.
# usage: tools/ab_bench.sh TAG LIB.so
set -o pipefail
TAG=${1:-ab}; LIB=$2
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.log
: > $OUT
row() {
  local label=$1; shift
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${TAG}_ab.tmp 2>&1 || { tail -5 gpurun_out/${TAG}_ab.tmp; exit 1; }
  python -c "
import json
r = json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); rf = r['roofline']
print('$label', r['config']['config'], r['config']['fit'], 'cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'], 4), 'pass_ms', round(rf['kernel_ms'], 4), 'ceiling_ms', round((rf.get('pattern_ceiling') or {}).get('ms', 0), 4))
" | tee -a $OUT
}
for rep in 1 2 3; do
  row new || exit 1
  PERT_LIB=$PWD/$LIB row old || exit 1
  row new --cells 1250 || exit 1
  PERT_LIB=$PWD/$LIB row old --cells 1250 || exit 1
  row new --fit step1 || exit 1
  PERT_LIB=$PWD/$LIB row old --fit step1 || exit 1
done
row new --config c5 || exit 1
PERT_LIB=$PWD/$LIB row old --config c5 || exit 1
