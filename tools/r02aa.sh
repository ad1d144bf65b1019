#!/bin/bash
# enum3 issue priority: falling by quarters (p1, default) vs none (p0), at 1,250 and 10k cells,
# interleaved, 2 reps, each line with its in-run ceiling; wave timelines of both at 1,250 cells
mkdir -p gpurun_out
R=$(pwd)
run() {
  local lib=$1; shift; local c=$1; shift
  PERT_LIB=$R/scdna_replication_tools_amd/ab_$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 3 --cells $c "$@" > gpurun_out/r02aa_b.log 2>&1 || return $?
  echo "$lib $c $(tail -1 gpurun_out/r02aa_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "frac_ceiling", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02aa_ab.log
}
for r in 1 2; do
  for lib in p1 p0; do
    run $lib 1250 || exit $?
    run $lib 10000 || exit $?
  done
done
for lib in st3 st3p0; do
  VARIANT=3 PERT_LIB=$R/scdna_replication_tools_amd/ab_$lib.so timeout -k 10 200 python tools/wave_timeline.py 1250 > gpurun_out/r02aa_timeline_$lib.log 2>&1 || exit $?
done
