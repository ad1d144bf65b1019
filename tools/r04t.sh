#!/bin/bash
# Short tiles for tiny one-rank shards (planner): the whole GPU suite (genome-length chain
# included), the C1 full fit and the C4 bench line (unchanged tiles there).
set -o pipefail
TAG=${1:-r04t}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_suite.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_suite.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python -u tools/fullfit_bench.py --config c1 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err || { tail -5 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/${TAG}_fullfit_c1.json').read().strip().splitlines()[-1])
t=d['timings_s']; print('C1 total', round(t['total'],3), 'ms_per_step', d['ms_per_step'], 'iters', d['iters'], 'acc', d.get('acc_cn'), d.get('acc_rep'))"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
