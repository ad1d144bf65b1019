#!/bin/bash
# full GPU suite on the current build, then C4 full fit (host stages), default bench, shard table
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02w_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02w_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02w_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02w_fullfit_c4.log
timeout -k 10 400 python bench.py > gpurun_out/r02w_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r02w_bench_default.log
for c in 10000 5000 2500 1250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 3 --cells $c > gpurun_out/r02w_b.log 2>&1 || exit $?
  echo "$c $(tail -1 gpurun_out/r02w_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02w_shards.log
done
