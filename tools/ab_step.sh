#!/bin/bash
# Step-time A/B of two builds (PERT_LIB) alternating on one box:
#   tools/ab_step.sh B.so "CELLS:LT ..." [rounds]
set -o pipefail
B=$1; SPECS=$2; R=${3:-2}
mkdir -p gpurun_out
for r in $(seq $R); do
  for spec in $SPECS; do
    set -- ${spec/:/ }
    for arm in A B; do
      if [ $arm = B ]; then export PERT_LIB=$(readlink -f $B); else unset PERT_LIB; fi
      timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --cells $1 --bins-per-tile $2 > gpurun_out/ab_$arm.log 2>&1 || exit 1
      python -c "
import json; r=json.loads(open('gpurun_out/ab_$arm.log').read().strip().splitlines()[-1]); print('$arm $1 $2', round(r['ms_per_step']*1e3,1), round(r['roofline']['kernel_ms']*1e3,1), round((r['ms_per_step']-r['roofline']['kernel_ms'])*1e3,1))"
    done
  done
done
