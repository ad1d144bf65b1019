#!/bin/bash
# Round-4 performance lease: roofline evidence of the headline pass (trace + PMC + bench
# --profile), the shard tile-length A/B, the C5 (20 kb) and step-1 bench lines.
set -o pipefail
TAG=${1:-r04f}
mkdir -p gpurun_out
bash tools/roofline_evidence.sh $TAG || exit 1
bash tools/shard_lt_ab.sh $TAG || exit 1
timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c5.log 2>&1 || { tail -5 gpurun_out/${TAG}_c5.log; exit 1; }
tail -1 gpurun_out/${TAG}_c5.log | cut -c1-600
timeout -k 10 200 python bench.py --fit step1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_step1.log 2>&1 || { tail -5 gpurun_out/${TAG}_step1.log; exit 1; }
tail -1 gpurun_out/${TAG}_step1.log | cut -c1-600
