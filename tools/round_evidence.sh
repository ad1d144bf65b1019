#!/bin/bash
# Round evidence on the GPU box (repo root): default bench (with cpu_baseline), then
# the rocprofv3 kernel-trace + PMC passes of tools/profile.sh.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench_default.log
timeout -k 10 1000 bash tools/profile.sh $TAG || exit 1
