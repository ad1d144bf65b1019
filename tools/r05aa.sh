#!/bin/bash
# pi-state placement search A/B: fresh processes, interleaved, PERT_PLACEMENT=0 (first allocation)
# vs the default search, C4 10 k and its 1,250-cell 8-GPU shard
set -o pipefail
TAG=${1:-r05aa}
mkdir -p gpurun_out
S="import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; pc=r.get('pattern_ceiling',{}); pl=r.get('pi_placement',{}); print('%-6s %5d ms/step %.4f kernel %.4f ceil %.4f value %.4g place %s' % (sys.argv[2], d['config']['cells'], d['ms_per_step'], r.get('kernel_ms') or 0, pc.get('ms') or 0, d['value'], pl.get('candidates_ms')))"
for rep in 1 2 3; do
  for pl in 0 4; do
    for c in "" "--cells 1250 --comm rccl"; do
      PERT_PLACEMENT=$pl timeout -k 10 200 python bench.py --no-cpu-baseline $c > gpurun_out/${TAG}.tmp 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
      tail -1 gpurun_out/${TAG}.tmp >> gpurun_out/${TAG}_bench.jsonl
      python3 -c "$S" gpurun_out/${TAG}.tmp "pl=$pl" | tee -a gpurun_out/${TAG}_ab.log
    done
  done
done
