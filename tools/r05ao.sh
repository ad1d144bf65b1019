#!/bin/bash
# Round 5, lease ao: full fits at HEAD -- C2 (clone_col=None: clustering + assignment first), C1
# in a fresh process (bench.py --fullfit-c1), C3 (2,000 cells, one GPU).
set -o pipefail
TAG=${1:-r05ao}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fullfit_bench.py --config c2 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c2.json 2> gpurun_out/${TAG}_fullfit_c2.err || { tail -5 gpurun_out/${TAG}_fullfit_c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c2.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('c2 total', t['total'], 'cluster_assign', t.get('cluster_assign'), 'phases', t['phases'][-1], 'acc', d.get('acc_cn'), d.get('acc_rep'), d.get('clusters_match_truth'))"
timeout -k 10 300 python -u tools/fullfit_bench.py --config c3 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c3.json 2> gpurun_out/${TAG}_fullfit_c3.err || { tail -5 gpurun_out/${TAG}_fullfit_c3.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c3.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('c3 total', t['total'], 'ms/step', d['ms_per_step'], 'iters', d['iters'])"
timeout -k 10 300 python -u bench.py --fullfit-c1 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err || { tail -5 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
tail -c 700 gpurun_out/${TAG}_fullfit_c1.json
