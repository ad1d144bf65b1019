#!/bin/bash
# several z / m / v sets in ONE process: fast and slow placements side by side?
set -o pipefail
TAG=${1:-r05z}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { echo "# $*" >> gpurun_out/${TAG}_sets.log; timeout -k 5 120 $P "$@" | tee -a gpurun_out/${TAG}_sets.log || exit 1; }
run 10000 5451 18 12 10 1 2 0 0 0 0 0 10000 12
run 1250 5451 54 12 20 1 2 0 0 0 0 0 1250 24
run 10000 5451 18 12 10 1 2 0 0 2 0 0 10000 8
run 1250 5451 54 12 20 1 2 0 0 2 0 0 1250 16
