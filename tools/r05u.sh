#!/bin/bash
# contiguous allocations: allocation size vs the small shard's ceiling (fresh process per run)
set -o pipefail
TAG=${1:-r05u}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { echo "# $*" >> gpurun_out/${TAG}_alloc.log; timeout -k 5 60 $P "$@" | tee -a gpurun_out/${TAG}_alloc.log || exit 1; }
for rep in 1 2 3; do
  run 1250 5451 54 12 20 1 2 0 0 2 0 0 10000
  run 1250 5451 54 12 20 1 2 0 0 2 0 0 1250
  run 1250 5451 54 12 20 1 2 0 0 0 0 0 10000
  run 2500 5451 54 12 20 1 2 0 0 2 0 0 2500
  run 5000 5451 36 12 20 1 2 0 0 2 0 0 5000
  run 10000 5451 18 12 20 1 2 0 0 2 0 0 10000
  run 10000 5451 18 12 20 1 2 0 0 0 0 0 10000
done
