#!/bin/bash
# placement search with the top-rate stop: where the 10 k and 1,250-cell searches end, and the set-up time
set -o pipefail
TAG=${1:-r05bu}
mkdir -p gpurun_out
for rep in 1 2 3 4; do
  for c in "" "--cells 1250 --comm rccl"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); r=d['roofline']; p=r['pi_placement']
print('%5d value-run %.4f kernel %.4f ceil %.4f tries %s' % (d['config']['cells'], d['ms_per_step'], r['kernel_ms'], r['pattern_ceiling']['ms'], p.get('candidates_ms')))" | tee -a gpurun_out/${TAG}_ab.log
  done
done
