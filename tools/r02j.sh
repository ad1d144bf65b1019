#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_loop.py tests/test_gpu_multirank.py tests/test_gpu_fit.py tests/test_gpu_chain.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02j_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/r02j_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
export PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_pk2.so
for r in 1 2; do
for c in 10000 1250; do
for a in "--variant 3" "--variant 3 --no-fused" "--variant 0"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c $a > gpurun_out/r02j_b.log 2>&1 || exit $?
  echo "$r $c $a $(tail -1 gpurun_out/r02j_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02j_ab.log
done
done
done
