#!/bin/bash
# tile order: XCD-aware bin-fastest (default, 2) vs XCD-aware cell-fastest (3) vs 2-D (0), on fast placements (the search on)
set -o pipefail
TAG=${1:-r05bh}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); print('%-10s %5d ms/step %.4f kernel %.4f ceil %.4f' % (sys.argv[2], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0))"
for rep in 1 2; do
  for lib in default tools/_ord3.so tools/_ord0.so; do
    for c in "--cells 1250 --comm rccl" ""; do
      if [ $lib = default ]; then unset PERT_LIB; else export PERT_LIB=$lib; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
      python3 -c "$S" gpurun_out/${TAG}.tmp "$(basename $lib)" | tee -a gpurun_out/${TAG}_ab.log
    done
  done
done
