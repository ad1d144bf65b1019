#!/bin/bash
# one allocation timed over 2 s (no new allocations), after a process that freed ~100 GB
set -o pipefail
TAG=${1:-r05af}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { echo "# $*" >> gpurun_out/${TAG}_watch.log; timeout -k 5 120 $P "$@" | tee -a gpurun_out/${TAG}_watch.log || exit 1; }
run 10000 5451 18 12 10 1 2 0 0 0 0 0 10000 1 100
run 10000 5451 18 12 10 1 2 0 0 0 0 0 10000 12
run 1250 5451 54 12 20 1 2 0 0 0 0 0 1250 1 100
