#!/bin/bash
# full fits on the final code: configs[0] stand-in (GPU vs measured CPU oracle chain), C2 stand-in
# (polyclonal, clone_col=None), C3
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --fullfit-c1 > gpurun_out/r02ae_fullfit_c1.log 2>&1 || exit $?
tail -1 gpurun_out/r02ae_fullfit_c1.log
timeout -k 10 600 python tools/fullfit_bench.py --config c2 --cpu-sample-cells 0 > gpurun_out/r02ae_fullfit_c2.log 2>&1 || exit $?
tail -1 gpurun_out/r02ae_fullfit_c2.log
timeout -k 10 600 python tools/fullfit_bench.py --config c3 --cpu-sample-cells 0 > gpurun_out/r02ae_fullfit_c3.log 2>&1 || exit $?
tail -1 gpurun_out/r02ae_fullfit_c3.log
timeout -k 10 600 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r02ae_fullfit_c4.log 2>&1 || exit $?
tail -1 gpurun_out/r02ae_fullfit_c4.log
