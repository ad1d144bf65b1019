#!/bin/bash
# one physically contiguous block for z / m / v with pads between them (exact relative physical
# offsets): does any offset give the fast pattern ceiling at 1,250 cells and at 10 k?
set -o pipefail
TAG=${1:-r05y}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { timeout -k 5 60 $P "$@" | tee -a gpurun_out/${TAG}_pads.log || exit 1; }
for rep in 1 2; do
  for pads in "0 0" "4 4" "64 64" "256 512" "1024 1024" "2048 2048" "2052 2052" "3072 3072" "8192 16384" "1024 3072"; do
    run 1250 5451 54 12 20 1 2 0 0 3 $pads
  done
  for pads in "0 0" "64 64" "1024 1024" "2048 2048" "2052 2052" "8192 16384"; do
    run 10000 5451 18 12 20 1 2 0 0 3 $pads
  done
done
