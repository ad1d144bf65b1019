#!/bin/bash
# low-coverage NB path in packed fp32 (shifted pairs, hoisted asymptotic pairs): C5 and C4 step
# times, then the GPU tests that cover the path (edge cases, configs incl. the C5 shard, parity)
set -o pipefail
TAG=${1:-r05as}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); print('%-14s %5d ms/step %.4f kernel %.4f ceil %.4f value %.4g' % (sys.argv[2], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0, d['value']))"
for c in "--config c5 --cells 250 --comm rccl" "--config c5" "" "--cells 1250 --comm rccl"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "$S" gpurun_out/${TAG}.tmp "$c" | tee -a gpurun_out/${TAG}_bench.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log
exit $rc
