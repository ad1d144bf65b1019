#!/bin/bash
# C2 pre-fit after the matrix-product assignment and the block consensus: profile, full fit, and
# the GPU tests through scRT (fit, chain)
set -o pipefail
TAG=${1:-r05au}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c2_profile.py --cprofile gpurun_out/${TAG}_c2.prof > gpurun_out/${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_c2.log; exit 1; }
tail -3 gpurun_out/${TAG}_c2.log
timeout -k 10 300 python -u tools/fullfit_bench.py --config c2 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c2.json 2> gpurun_out/${TAG}_fullfit_c2.err || { tail -5 gpurun_out/${TAG}_fullfit_c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c2.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('c2 total', t['total'], 'cluster_assign', t.get('cluster_assign'), 'acc', d.get('acc_cn'), d.get('acc_rep'), d.get('clusters_match_truth'))"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fit.py tests/test_gpu_chain.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log
exit $rc
