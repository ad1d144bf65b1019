#!/bin/bash
# Standard GPU round: parity tests, then benches (both enumerated-pass variants).
# usage (on the box, repo root): tools/gpu_check.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench_v0.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench_v0.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --variant 1 "$@" > gpurun_out/${TAG}_bench_v1.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench_v1.log
