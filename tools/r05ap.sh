#!/bin/bash
# one-launch step (pert_enum_step) vs the three-launch step at 10 k cells, fast placements
set -o pipefail
TAG=${1:-r05ap}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); pl=r.get('pi_placement',{}); print('%-9s %5d ms/step %.4f kernel %.4f ceil %.4f value %.4g place %s' % (sys.argv[2], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0, d['value'], pl.get('candidates_ms')))"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_placement.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for rep in 1 2 3; do
  for f in "--no-fused" "--fused"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $f > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "$S" gpurun_out/${TAG}.tmp "$f" | tee -a gpurun_out/${TAG}_ab.log
  done
done
