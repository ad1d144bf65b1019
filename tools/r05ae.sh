#!/bin/bash
# small shard inside larger allocations: 1,250 cells launched over z / m / v sets sized for 10 k /
# 5 k / 1,250 cells (several sets per process, each held): how often is the set fast?
set -o pipefail
TAG=${1:-r05ae}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { echo "# $*" >> gpurun_out/${TAG}_sets.log; timeout -k 5 120 $P "$@" | tee -a gpurun_out/${TAG}_sets.log || exit 1; }
run 1250 5451 54 12 20 1 2 0 0 0 0 0 10000 12
run 1250 5451 54 12 20 1 2 0 0 0 0 0 5000 16
run 1250 5451 54 12 20 1 2 0 0 0 0 0 1250 40
run 10000 5451 18 12 10 1 2 0 0 0 0 0 10000 8
