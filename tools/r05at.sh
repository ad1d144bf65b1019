#!/bin/bash
# low-coverage NB path A/B: HEAD's math (v0), packed shift pairs + hoisted pairs (v1, in-tree),
# v1 with two waves per SIMD (no spills): C5 and C4 shards
set -o pipefail
TAG=${1:-r05at}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); print('%-12s %-34s %5d LT %s ms/step %.4f kernel %.4f ceil %.4f' % (sys.argv[2], sys.argv[3], d['config']['cells'], d['config']['bins_per_tile'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0))"
for lib in tools/_v0.so default tools/_v1w2.so; do
  for c in "--config c5 --cells 250 --comm rccl" "--config c5" "--cells 1250 --comm rccl" ""; do
    if [ $lib = default ]; then unset PERT_LIB; else export PERT_LIB=$lib; fi
    timeout -k 10 240 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "$S" gpurun_out/${TAG}.tmp "$(basename $lib)" "$c" | tee -a gpurun_out/${TAG}_ab.log
  done
done
