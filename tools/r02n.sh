#!/bin/bash
# HBM ceilings (read-only / write-only / copy) and variant-3 tile-length A/B at 1,250 and 10k cells
mkdir -p gpurun_out
timeout -k 10 120 ./tools/stream_probe 10000 5451 48 20 > gpurun_out/r02n_probe.log 2>&1 || exit $?
for c in 1250 10000; do
for a in "--variant 3 --no-fused" "--variant 3"; do
for lt in 0 12 18 27 36 54; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 3 --cells $c --bins-per-tile $lt $a > gpurun_out/r02n_b.log 2>&1 || exit $?
  echo "$c $a lt=$lt $(tail -1 gpurun_out/r02n_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02n_ab.log
done
done
done
