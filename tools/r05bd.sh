#!/bin/bash
# Round 5, lease bd: at HEAD -- C1 in a fresh process (bench.py --fullfit-c1), C2 and C4 full fits
set -o pipefail
TAG=${1:-r05bd}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --fullfit-c1 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err || { tail -5 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c1.json').read().strip().splitlines()[-1]); print('c1 gpu_s', d['gpu_s'], 'cpu', d['cpu_baseline']['seconds'], 'speedup', d['speedup'])"
for c in c2 c4; do
  timeout -k 10 300 python -u tools/fullfit_bench.py --config $c --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_$c.json 2> gpurun_out/${TAG}_fullfit_$c.err || { tail -5 gpurun_out/${TAG}_fullfit_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_$c.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('$c total', t['total'], 'cluster_assign', t.get('cluster_assign'), 'iters', d['iters'], 'acc', d.get('acc_cn'), d.get('acc_rep'))"
done
