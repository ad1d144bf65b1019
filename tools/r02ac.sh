#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -v -s --timeout 170 --timeout-method thread -k run_pert_model tests/test_gpu_zz_api_ranks.py > gpurun_out/r02ac_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02ac_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02ac_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02ac_fullfit_c4.log
