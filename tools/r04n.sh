#!/bin/bash
# Step-1 / shard tile-length sweep (tools/r04n_sweep.sh), the write-through store A/B, and the
# step-1 GPU tests at the new tile limit.
set -o pipefail
TAG=${1:-r04n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_parity.py -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "step1" > gpurun_out/${TAG}_s1tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_s1tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_s1tests.log
bash tools/r04n_sweep.sh $TAG || exit 1
bash tools/ab_bench.sh ${TAG}_cpol19 ab/libpert_cpol19.so || exit 1
