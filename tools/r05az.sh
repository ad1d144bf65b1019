#!/bin/bash
# sorted input tables deferred to a background thread: C4 full fit timeline, then the GPU tests
# through run_pert_model (chain, fit, two-rank API)
set -o pipefail
TAG=${1:-r05az}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -5 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c4.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('c4 total', t['total'], 'phases', t['phases'], 'iters', d['iters'], 'acc', d.get('acc_cn'), d.get('acc_rep'))"
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_fit.py tests/test_gpu_zz_api_ranks.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log
exit $rc
