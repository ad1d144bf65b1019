#!/bin/bash
# after the placement-search change: its GPU tests, then the C4 full fit twice
set -o pipefail
TAG=${1:-r05bv}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_placement.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -2
for rep in 1 2; do
  timeout -k 10 600 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c4_$rep.json 2> gpurun_out/${TAG}_fullfit_c4_$rep.err || { tail -20 gpurun_out/${TAG}_fullfit_c4_$rep.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c4_$rep.json').read().strip().splitlines()[-1])
print({k: d[k] for k in d if k in ('total_s','wall_s','gpu_s','ms_per_step','iterations','timings_s')} or list(d)[:20])"
done
