#!/bin/bash
# Round 5, lease c: GPU suite (enum_jmax without the scale factor: the chain's stops), the
# bytes-in-flight probe at the 1,250-cell shard, and the pass vs its ceiling over tile lengths.
set -o pipefail
TAG=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
python -c "
import json; d=json.load(open('gpurun_out/parity_report.json')); g=d.get('genome_chain_64x64x5451',{})
print('chain stops', g.get('stops'))"
for args in "1250 5451 54 12" "1250 5451 54 8" "1250 5451 42 12" "1250 5451 36 12" "1250 5451 27 12" "1250 5451 18 12" \
            "10000 5451 18 12" "10000 5451 54 12"; do
  timeout -k 5 60 ./tools/depth_probe $args 20 | tee -a gpurun_out/${TAG}_depth.log || exit 1
done
for lt in 54 42 36 27; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --cells 1250 --comm rccl --no-cpu-baseline \
    --bins-per-tile $lt > gpurun_out/${TAG}_bench.tmp 2>&1 || { cat gpurun_out/${TAG}_bench.tmp; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_bench.tmp | tee -a gpurun_out/${TAG}_bench.jsonl | python -c "
import json,sys
r=json.loads(sys.stdin.read()); rf=r['roofline']
print(r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'ms/step %.4f' % r['ms_per_step'], 'noev %.4f' % r.get('ms_per_step_no_events', -1),
      'kernel %.4f' % rf['kernel_ms'], 'ceil %.4f' % rf['pattern_ceiling']['ms'])"
done
