#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_loop.py tests/test_gpu_multirank.py -m gpu -v --timeout 200 --timeout-method thread -s > gpurun_out/r02h_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/r02h_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
for r in 1 2; do
for a in "--variant 3" "--variant 3 --no-fused" "--variant 0"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 3 $a > gpurun_out/r02h_b.log 2>&1 || exit $?
  echo "$r $a $(tail -1 gpurun_out/r02h_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02h_ab.log
done
done
