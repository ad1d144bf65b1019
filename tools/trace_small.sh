#!/bin/bash
# kernel traces of the default bench and of a small shard (the per-rank work of an
# 8-GPU strong-scaling run), plus the GPU tests
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/trace_small gpurun_out/trace_c4
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_small -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --cells 1250 --steps 30 > $R/gpurun_out/trace_small/log.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_c4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 > $R/gpurun_out/trace_c4/log.txt 2>&1 || exit 1
echo traced
