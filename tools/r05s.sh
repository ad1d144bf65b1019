#!/bin/bash
# placement of z / m / v and the tile length: the pattern's ceiling (depth_probe, order 2)
set -o pipefail
TAG=${1:-r05s}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { timeout -k 5 60 $P "$@" | tee -a gpurun_out/${TAG}_placement.log || exit 1; }
for rep in 1 2; do
  run 10000 5451 18 12 20 1 2
  run 10000 5451 54 12 20 1 2
  run 10000 5451 54 12 20 1 2 0 20
  run 1250 5451 54 12 20 1 2
  run 1250 5451 18 12 20 1 2
  for pads in "0 0" "4 4" "64 64" "1024 2048" "2052 4104" "16384 32768" "65536 131072" "262144 524288" "1048576 2097152" "2801664 2801664"; do
    run 1250 5451 54 12 20 1 2 0 0 1 $pads
  done
  run 10000 5451 18 12 20 1 2 0 0 1 0 0
  run 10000 5451 54 12 20 1 2 0 0 1 0 0
done
