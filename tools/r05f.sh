#!/bin/bash
# Round 5, lease f: the three-wave pass's workgroup -> tile order (PERT_ENUM3_ORDER 0..3), probe
# and interleaved bench A/B at C4 (10 k cells) and the 1,250-cell shard, one box.
set -o pipefail
TAG=${1:-r05f}
mkdir -p gpurun_out
: > gpurun_out/${TAG}_orders.log
for args in "10000 5451 18 12 20 1 0" "10000 5451 18 12 20 1 1" "10000 5451 18 12 20 1 2" "10000 5451 18 12 20 1 3" \
            "1250 5451 54 12 20 1 0" "1250 5451 54 12 20 1 2" "1250 5451 54 12 20 1 3"; do
  timeout -k 5 60 ./tools/depth_probe $args | tee -a gpurun_out/${TAG}_depth.log || exit 1
done
row() {
  local label=$1; shift
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${TAG}_b.tmp 2>&1 \
    || { tail -5 gpurun_out/${TAG}_b.tmp; exit 1; }
  python -c "
import json
r = json.loads(open('gpurun_out/${TAG}_b.tmp').read().strip().splitlines()[-1]); rf = r['roofline']
print('$label cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms %.4f' % r['ms_per_step'], 'pass_ms %.4f' % rf['kernel_ms'], 'ceiling_ms %.4f' % rf['pattern_ceiling']['ms'], 'frac %.3f' % rf['frac'])
" | tee -a gpurun_out/${TAG}_orders.log
}
for rep in 1 2; do
  row order0
  PERT_LIB=$PWD/ab/libpert_order1.so row order1
  PERT_LIB=$PWD/ab/libpert_order2.so row order2
  PERT_LIB=$PWD/ab/libpert_order3.so row order3
  row order0 --cells 1250 --comm rccl
  PERT_LIB=$PWD/ab/libpert_order1.so row order1 --cells 1250 --comm rccl
  PERT_LIB=$PWD/ab/libpert_order2.so row order2 --cells 1250 --comm rccl
  PERT_LIB=$PWD/ab/libpert_order3.so row order3 --cells 1250 --comm rccl
done
