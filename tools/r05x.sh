#!/bin/bash
# wave timeline at 1,250 cells (54 bins): variance by XCD / CU / SIMD, raw stamps kept
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  PERT_LIB=tools/_stamps.so VARIANT=3 LT=54 DUMP=gpurun_out/r05x_stamps_$rep.npz timeout -k 10 120 python tools/wave_timeline.py 1250 >> gpurun_out/r05x_timeline.log 2>&1 || exit 1
done
grep -E "span|share|exit" gpurun_out/r05x_timeline.log
timeout -k 10 120 python tools/rccl_two_ranks.py > gpurun_out/r05x_rccl_two_ranks.log 2>&1; tail -3 gpurun_out/r05x_rccl_two_ranks.log
