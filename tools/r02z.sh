#!/bin/bash
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_chain.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02z_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02z_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02z_fullfit_c4.log
for c in 1250 10000; do
  VARIANT=3 PERT_LIB=$R/scdna_replication_tools_amd/ab_st3.so timeout -k 10 200 python tools/wave_timeline.py $c > gpurun_out/r02z_timeline_$c.log 2>&1 || exit $?
done
