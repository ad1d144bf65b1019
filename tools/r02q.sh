#!/bin/bash
# same-box tile-length A/B: variant 3 (separate finalize/adam) vs variant 0, interleaved, 2 reps;
# each line carries the in-run pattern ceiling (pert_stream_ceiling)
mkdir -p gpurun_out
run() {  # cells, label, args...
  local c=$1; shift; local lab=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c "$@" > gpurun_out/r02q_b.log 2>&1 || return $?
  echo "$c $lab $(tail -1 gpurun_out/r02q_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02q_ab.log
}
for r in 1 2; do
  for lt in 12 18 24 36 0; do run 10000 "v3nf lt=$lt" --variant 3 --no-fused --bins-per-tile $lt || exit $?; done
  run 10000 "v0 auto" --variant 0 || exit $?
  for lt in 12 18 27 43 54 64 0; do run 1250 "v3nf lt=$lt" --variant 3 --no-fused --bins-per-tile $lt || exit $?; done
  run 1250 "v0 auto" --variant 0 || exit $?
done
