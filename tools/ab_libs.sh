#!/bin/bash
# Step-time A/B of several builds (PERT_LIB; "-" = the in-tree library), alternating on one box:
#   tools/ab_libs.sh TAG "BENCH ARGS" rounds lib1 lib2 ...
set -o pipefail
TAG=$1; ARGS=$2; R=$3; shift 3
mkdir -p gpurun_out
for r in $(seq $R); do
  for L in "$@"; do
    if [ "$L" = - ]; then unset PERT_LIB; else export PERT_LIB=$(readlink -f $L); fi
    timeout -k 10 200 python bench.py --no-cpu-baseline $ARGS > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); r=d['roofline']
print('%-14s value-run %.4f evented-run %.4f kernel %.4f ceil %.4f' % ('$L', d['ms_per_step'], d['ms_per_step_evented'], r['kernel_ms'], r['pattern_ceiling']['ms']))" | tee -a gpurun_out/${TAG}_ab.log
  done
done
