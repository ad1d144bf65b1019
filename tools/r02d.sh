#!/bin/bash
# variant-3 (three-wave pass, fused step) GPU checks, then an A/B of variants 0 / 3 at C4.
# A crash / fault / time limit (exit >= 2 from pytest, >= 124 from anything) ends the script.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_loop.py \
  tests/test_gpu_fit.py tests/test_gpu_chain.py -m gpu -v --timeout 200 --timeout-method thread -s \
  > gpurun_out/r02d_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/r02d_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
bash tools/var_ab.sh "0 3" "10000" > gpurun_out/r02d_ab.log 2>&1
rc=$?
echo "ab exit $rc" >> gpurun_out/r02d_ab.log
exit $rc
