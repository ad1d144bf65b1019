#!/bin/bash
# Round 5, lease b: loader probe of a two-rank fit, fresh-process C1 profile, bench lines
# (C4; the 1,250-cell shard unsharded and with the library's RCCL all-reduce at world 1).
set -o pipefail
TAG=${1:-r05b}
mkdir -p gpurun_out
timeout -k 10 280 python -u tools/dl_probe.py --world2 > gpurun_out/${TAG}_dlprobe.log 2>&1; rc=$?
tail -30 gpurun_out/${TAG}_dlprobe.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -m pytest tests/test_gpu_zz_api_ranks.py tests/test_gpu_native_comm.py -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/c1_fresh.py --cprofile gpurun_out/${TAG}_c1.prof --repeat 1 > gpurun_out/${TAG}_c1.json 2> gpurun_out/${TAG}_c1.err || exit 1
cat gpurun_out/${TAG}_c1.json | cut -c1-600
for rep in 1 2; do
  for cfg in "" "--cells 1250" "--cells 1250 --comm rccl"; do
    echo "== bench $cfg (rep $rep)"
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 $cfg $( [ -n "$cfg" ] && echo --no-cpu-baseline ) \
      > gpurun_out/${TAG}_bench.tmp 2>&1 || { cat gpurun_out/${TAG}_bench.tmp; exit 1; }
    grep '"metric"' gpurun_out/${TAG}_bench.tmp | tee -a gpurun_out/${TAG}_bench.jsonl | python -c "
import json,sys
r=json.loads(sys.stdin.read()); rf=r['roofline']
print(r['config']['cells'], 'ms/step %.4f' % r['ms_per_step'], 'noev %.4f' % r.get('ms_per_step_no_events', -1),
      'kernel %.4f' % rf['kernel_ms'], 'ceil %.4f' % rf['pattern_ceiling']['ms'], 'frac %.3f' % rf['frac'], r['config']['allreduce'][:20])"
  done
done
