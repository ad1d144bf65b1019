#!/bin/bash
# C5 (20 kb bins): is the pass compute-bound on the low-coverage NB path?  Reads per cell 1e6
# (the config: D ~ 1.2, shift + direct pairs) vs 1e7 (D ~ 12: the hoisted asymptotic path)
set -o pipefail
TAG=${1:-r05ar}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); print('%-14s %5d ms/step %.4f kernel %.4f ceil %.4f value %.4g' % (sys.argv[2], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0, d['value']))"
for rpc in 1e6 1e7; do
  for c in "--cells 250 --comm rccl" ""; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --config c5 --reads-per-cell $rpc $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "$S" gpurun_out/${TAG}.tmp "reads=$rpc" | tee -a gpurun_out/${TAG}_c5.log
  done
done
