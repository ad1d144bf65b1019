#!/bin/bash
# is the helper's slowdown of the step numpy's BLAS thread pool?  helper-load with OPENBLAS_NUM_THREADS=1
# vs default, alternating; then the C4 full fit with OPENBLAS_NUM_THREADS=1
set -o pipefail
TAG=${1:-r05bz}
mkdir -p gpurun_out
python3 -c "import threadpoolctl, numpy; print([(d['internal_api'], d['num_threads'], d['filepath'].split('/')[-1]) for d in threadpoolctl.threadpool_info()])" | tee gpurun_out/${TAG}_pools.log
for rep in 1 2; do
  for e in "" "OPENBLAS_NUM_THREADS=1"; do
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --cells 1250 --comm rccl --helper-load > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); r=d['roofline']
print('%-24s value-run %.4f evented-run %.4f kernel %.4f helper %s' % ('$e', d['ms_per_step'], d['ms_per_step_evented'], r['kernel_ms'], (d.get('helper_load') or {}).get('cells_per_s')))" | tee -a gpurun_out/${TAG}_ab.log
  done
done
OPENBLAS_NUM_THREADS=1 timeout -k 10 600 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -20 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_fullfit_c4.json').read().strip().splitlines()[-1]); t=d['timings_s']
print('fullfit total', t['total'], t['phases'], t['ms_per_step'] if 'ms_per_step' in t else d.get('ms_per_step'))"
