#!/bin/bash
# variant-3 tile length at the 2- and 4-rank shards of C4 (5,000 / 2,500 cells), 2 reps
mkdir -p gpurun_out
run() {
  local c=$1; shift; local lab=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c "$@" > gpurun_out/r02r_b.log 2>&1 || return $?
  echo "$c $lab $(tail -1 gpurun_out/r02r_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02r_ab.log
}
for r in 1 2; do
  for c in 2500 5000; do
    for lt in 12 18 27 36 43 54 64; do run $c "v3nf lt=$lt" --variant 3 --no-fused --bins-per-tile $lt || exit $?; done
  done
done
# C5 (2k cells x 136,275 20 kb bins): variant 0 vs variant 3
for a in "v0 --variant 0" "v3nf --variant 3 --no-fused" "v3nf18 --variant 3 --no-fused --bins-per-tile 18" "v3nf43 --variant 3 --no-fused --bins-per-tile 43"; do
  set -- $a; lab=$1; shift
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/r02r_c5.log 2>&1 || exit $?
  echo "c5 $lab $(tail -1 gpurun_out/r02r_c5.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "frac", round(r["frac"],3), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02r_ab.log
done
