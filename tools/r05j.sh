#!/bin/bash
# Round 5, lease j: load schedule with arithmetic in between (depth_probe work mode): m / v in the
# bin that uses them (the pass's schedule) or a bin ahead, at 1,250 and 10 k cells.
set -o pipefail
TAG=${1:-r05j}
mkdir -p gpurun_out
timeout -k 5 60 ./tools/depth_probe 10000 5451 18 12 20 1 2 | tee -a gpurun_out/${TAG}_work.log || exit 1
for w in 400 800 1600; do
  for args in "1250 5451 54 12" "1250 5451 54 8" "10000 5451 18 12" "10000 5451 18 8"; do
    timeout -k 5 60 ./tools/depth_probe $args 20 1 2 $w | tee -a gpurun_out/${TAG}_work.log || exit 1
  done
done
