#!/bin/bash
# Round 5, lease e: loop tests (events now recorded inside pert_svi_run), the footprint / grid-order
# probe of the small-shard ceiling, the bench line with an event-free value region, and the
# planner's 67-85 %-of-slots band (1,600 cells) A/B.
set -o pipefail
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_loop.py tests/test_gpu_native_comm.py -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for args in "10000 5451 18 12 20 1 0" "1250 5451 54 12 20 1 0" "1250 5451 54 12 20 8 0" "1250 5451 54 12 20 1 1" \
            "1250 5451 54 12 20 8 1" "2500 5451 12 12 20 1 0" "2500 5451 12 12 20 4 0" "10000 5451 18 12 20 1 1"; do
  timeout -k 5 60 ./tools/depth_probe $args | tee -a gpurun_out/${TAG}_depth.log || exit 1
done
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_bench.log | python -c "
import json,sys; r=json.loads(sys.stdin.read()); rf=r['roofline']
print('C4 value %.4g ms/step %.4f evented %.4f kernel %.4f ceil %.4f frac %.3f cpu %.4g' % (r['value'], r['ms_per_step'], r['ms_per_step_evented'], rf['kernel_ms'], rf['pattern_ceiling']['ms'], rf['frac'], r['cpu_baseline']['value']))"
for rep in 1 2; do
  for lt in 0 53 64 18; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --cells 1600 --comm rccl --no-cpu-baseline \
      --bins-per-tile $lt > gpurun_out/${TAG}_b.tmp 2>&1 || { cat gpurun_out/${TAG}_b.tmp; exit 1; }
    grep '"metric"' gpurun_out/${TAG}_b.tmp | tee -a gpurun_out/${TAG}_planner.jsonl | python -c "
import json,sys; r=json.loads(sys.stdin.read()); rf=r['roofline']
print(r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'ms/step %.4f' % r['ms_per_step'], 'kernel %.4f ceil %.4f' % (rf['kernel_ms'], rf['pattern_ceiling']['ms']))"
  done
done
