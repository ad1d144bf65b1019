#!/bin/bash
# helper-load at K = 200 steps (a longer C call: the interpreter-lock hand-offs at its two ends weigh 10x less)
set -o pipefail
TAG=${1:-r05ca}
mkdir -p gpurun_out
for rep in 1 2; do
  for c in "" "--helper-load"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --cells 1250 --comm rccl --steps 200 $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); r=d['roofline']
print('K=200 %-14s value-run %.4f evented-run %.4f kernel %.4f helper %s' % ('$c', d['ms_per_step'], d['ms_per_step_evented'], r['kernel_ms'], (d.get('helper_load') or {}).get('cells_per_s')))" | tee -a gpurun_out/${TAG}_ab.log
  done
done
