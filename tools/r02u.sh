#!/bin/bash
# finalize loads in flight (4 vs 8 bin tiles per thread) at 10k (LT 12 / 18) and 1,250 cells;
# then the streaming ceiling vs bytes at 1,250 cells (fixed per-launch cost?)
mkdir -p gpurun_out
R=$(pwd)
run() {
  local lib=$1; shift; local c=$1; shift; local lab=$1; shift
  PERT_LIB=$R/scdna_replication_tools_amd/ab_$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 3 --cells $c "$@" > gpurun_out/r02u_b.log 2>&1 || return $?
  echo "$lib $c $lab $(tail -1 gpurun_out/r02u_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_ms", round(r["pattern_ceiling"]["ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02u_ab.log
}
for r in 1 2; do
  for lib in fin4 fin8; do
    run $lib 10000 lt12 --bins-per-tile 12 || exit $?
    run $lib 10000 lt18 --bins-per-tile 18 || exit $?
    run $lib 1250 auto || exit $?
  done
  run fin4 1250 fused --fused || exit $?
  run fin4 10000 fused --fused || exit $?
done
for b in 5451 10902 21804; do
  timeout -k 10 200 ./tools/stream_probe 1250 $b 43 20 2>&1 | grep "separate hipMalloc" | sed "s/^/1250 x $b: /" >> gpurun_out/r02u_probe.log || exit $?
done
for c in 2500 5000 10000; do
  timeout -k 10 200 ./tools/stream_probe $c 5451 12 10 2>&1 | grep "separate hipMalloc" | sed "s/^/$c x 5451: /" >> gpurun_out/r02u_probe.log || exit $?
done
