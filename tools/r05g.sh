#!/bin/bash
# Round 5, lease g: GPU suite with the XCD-aware tile order as default, the default bench line,
# the shard table, the per-rank host work of a two-rank fit at 2,000 + 2,000 cells x 5,451 bins.
set -o pipefail
TAG=${1:-r05g}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
python -c "
import json; d=json.load(open('gpurun_out/parity_report.json')); g=d.get('genome_chain_64x64x5451',{})
print('chain stops', {k: v['product'] for k, v in g.get('stops', {}).items()})"
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_bench.log | python -c "
import json,sys; r=json.loads(sys.stdin.read()); rf=r['roofline']
print('C4 value %.4g ms/step %.4f evented %.4f kernel %.4f ceil %.4f frac %.3f cpu %.4g' % (r['value'], r['ms_per_step'], r['ms_per_step_evented'], rf['kernel_ms'], rf['pattern_ceiling']['ms'], rf['frac'], r['cpu_baseline']['value']))"
rm -f gpurun_out/${TAG}_shards.jsonl
for rep in 1 2; do
  for cfg in "--cells 10000" "--cells 1250 --comm rccl" "--cells 2500 --comm rccl" "--cells 5000 --comm rccl"; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $cfg > gpurun_out/${TAG}_b.tmp 2>&1 \
      || { cat gpurun_out/${TAG}_b.tmp; exit 1; }
    grep '"metric"' gpurun_out/${TAG}_b.tmp | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_fused']=False
print(json.dumps(r))" >> gpurun_out/${TAG}_shards.jsonl
  done
done
python tools/shard_table.py gpurun_out/${TAG}_shards.jsonl | tee gpurun_out/${TAG}_shard_sizes.log
timeout -k 10 500 python -u tools/api_ranks_timing.py --cells 2000 --max-iter 200 > gpurun_out/${TAG}_api_ranks.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_api_ranks.log; exit 1; }
tail -1 gpurun_out/${TAG}_api_ranks.log
