set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_tau.py -x -v -s --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03k_tau_tests.log 2>&1 || { tail -40 gpurun_out/r03k_tau_tests.log; exit 1; }
grep -E "PASSED|FAILED|percentile|guess_times|C1-size" gpurun_out/r03k_tau_tests.log
timeout -k 10 240 python -u tools/tau_probe.py > gpurun_out/r03k_tau_probe.log 2>&1 || { tail -20 gpurun_out/r03k_tau_probe.log; exit 1; }
cat gpurun_out/r03k_tau_probe.log
