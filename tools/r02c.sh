set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py tests/test_gpu_chain.py -m gpu -x -v --timeout 200 --timeout-method thread -s > gpurun_out/r02c_tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/r02c_tests.log
bash tools/var_ab.sh "0 3" "10000" > gpurun_out/r02c_ab.log 2>&1
echo "ab exit $?" >> gpurun_out/r02c_ab.log
