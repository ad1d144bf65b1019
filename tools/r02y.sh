#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_chain.py tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02y_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02y_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02y_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02y_fullfit_c4.log
timeout -k 10 600 python tools/host_prep_cprofile.py > gpurun_out/r02y_hostprep.log 2>&1 || exit $?
