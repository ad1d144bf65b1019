set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 || exit 1
tail -1 gpurun_out/b_default.log | cut -c1-400
for LT in 16 64; do timeout -k 10 200 python bench.py --no-cpu-baseline --bins-per-tile $LT > gpurun_out/b_lt$LT.log 2>&1 || exit 1; echo LT$LT; tail -1 gpurun_out/b_lt$LT.log | cut -c1-300; done
for LT in 8 16 32; do timeout -k 10 200 python bench.py --no-cpu-baseline --cells 1250 --bins-per-tile $LT > gpurun_out/b_1250_lt$LT.log 2>&1 || exit 1; echo 1250 LT$LT; tail -1 gpurun_out/b_1250_lt$LT.log | cut -c1-300; done
