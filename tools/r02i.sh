#!/bin/bash
mkdir -p gpurun_out
export PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_pk.so
for r in 1 2; do
for c in 10000 1250; do
for a in "--variant 3" "--variant 3 --no-fused" "--variant 0"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c $a > gpurun_out/r02i_b.log 2>&1 || exit $?
  echo "$r $c $a $(tail -1 gpurun_out/r02i_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02i_ab.log
done
done
done
