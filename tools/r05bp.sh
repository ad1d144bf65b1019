#!/bin/bash
# the one-launch step (pert_enum_step) vs three launches on the small sharded shards, alternating
set -o pipefail
TAG=${1:-r05bp}
mkdir -p gpurun_out
for rep in 1 2 3; do
  for c in "--cells 1250 --comm rccl" "--cells 1250 --comm rccl --fused" "--cells 2500 --comm rccl" "--cells 2500 --comm rccl --fused"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); r=d['roofline']
print('%-40s value-run %.4f evented-run %.4f kernel %.4f ceil %.4f' % ('$c', d['ms_per_step'], d['ms_per_step_evented'], r['kernel_ms'], r['pattern_ceiling']['ms']))" | tee -a gpurun_out/${TAG}_ab.log
  done
done
