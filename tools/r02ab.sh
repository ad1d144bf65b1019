#!/bin/bash
mkdir -p gpurun_out
R=$(pwd)
VARIANT=3 PERT_LIB=$R/scdna_replication_tools_amd/ab_st3.so timeout -k 10 200 python tools/wave_timeline.py 1250 > gpurun_out/r02ab_timeline_1250.log 2>&1 || exit $?
for c in 250 2000; do
  timeout -k 10 300 python bench.py --config c5 --cells $c --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r02ab_c5_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/r02ab_c5_$c.log
done
