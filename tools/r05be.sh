#!/bin/bash
# C1 in fresh processes, three times (first-use costs vary by box)
set -o pipefail
TAG=${1:-r05be}
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --fullfit-c1 > gpurun_out/${TAG}_fullfit_c1_$rep.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c1_$rep.json').read().strip().splitlines()[-1]); t=d['gpu_timings_s']
print('c1 gpu_s %.3f cpu %.2f speedup %.1f init1 %s step1 %.3f tau %s' % (d['gpu_s'], d['cpu_baseline']['seconds'], d['speedup'], t['init_shard1']['inputs'], t['step1'], t['tau_init_s']['batched_s']))"
done
