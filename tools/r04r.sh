#!/bin/bash
# One-launch steps for tiny single-rank fits (pert_model._fused): the chain tests (tutorial, C1,
# genome length) and the loop tests through it, then the C1 full fit with and without it.
set -o pipefail
TAG=${1:-r04r}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_loop.py tests/test_gpu_multirank.py -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|genome chain vs" gpurun_out/${TAG}_tests.log | cut -c1-600 | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for f in 0 auto; do
  PERT_FUSED=$f timeout -k 10 200 python -u tools/fullfit_bench.py --config c1 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c1_$f.json 2> gpurun_out/${TAG}_fullfit_c1_$f.err || { tail -5 gpurun_out/${TAG}_fullfit_c1_$f.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/${TAG}_fullfit_c1_$f.json').read().strip().splitlines()[-1])
t=d['timings_s']; print('PERT_FUSED=$f', 'total', round(t['total'],3), 'ms_per_step', d['ms_per_step'], 'iters', d['iters'])"
done
