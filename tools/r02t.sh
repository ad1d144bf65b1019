#!/bin/bash
# full fits (configs[0] stand-in: GPU vs measured CPU oracle chain; C4 end to end with host
# stages) and the per-rank shard table of C4's strong scaling on the default build
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --fullfit-c1 > gpurun_out/r02t_fullfit_c1.log 2>&1 || exit $?
tail -1 gpurun_out/r02t_fullfit_c1.log
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02t_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02t_fullfit_c4.log
for r in 1 2; do
for c in 10000 5000 2500 1250; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 3 --cells $c > gpurun_out/r02t_b.log 2>&1 || exit $?
  echo "$c $(tail -1 gpurun_out/r02t_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02t_shards.log
done
done
