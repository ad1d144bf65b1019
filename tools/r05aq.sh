#!/bin/bash
# tile length at 10 k cells on fast placements (the search on): does the planner's 54 still win?
set -o pipefail
TAG=${1:-r05aq}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); pl=r.get('pi_placement',{}); print('LT %3s %5d ms/step %.4f kernel %.4f ceil %.4f value %.4g place %s' % (d['config']['bins_per_tile'], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0, d['value'], pl.get('candidates_ms')))"
for rep in 1 2; do
  for lt in 18 27 36 54 12; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --bins-per-tile $lt > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "$S" gpurun_out/${TAG}.tmp | tee -a gpurun_out/${TAG}_lt.log
  done
done
