#!/bin/bash
# small-shard breakdown: per-kernel trace stats of bench.py at 1,250 cells, tile lengths 54 / 36 / 18, fused and not
set -o pipefail
TAG=${1:-r05v}
R=$(pwd)
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
i=0
for A in "--bins-per-tile 54" "--bins-per-tile 36" "--bins-per-tile 18" "--bins-per-tile 54 --fused" "--bins-per-tile 27" ; do
  i=$((i+1))
  echo "== $A" >> $R/gpurun_out/$TAG/summary.txt
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/t$i -o run --output-format csv -- \
    python3 $R/bench.py --cells 1250 --comm rccl --steps 40 --warmup 5 --no-cpu-baseline $A > $R/gpurun_out/$TAG/t$i.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/$TAG/t$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'noev', d.get('ms_per_step_no_events'), 'roof', {k: d['roofline'].get(k) for k in ('kernel_ms','ceiling_ms','frac_ceiling') if k in d['roofline']})" >> $R/gpurun_out/$TAG/summary.txt
  f=$(find $R/gpurun_out/$TAG/t$i -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('  %-60s calls %6s avg %10.1f us tot %8.2f %%' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['Percentage'])))" >> $R/gpurun_out/$TAG/summary.txt
done
cat $R/gpurun_out/$TAG/summary.txt
