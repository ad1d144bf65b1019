#!/bin/bash
# allocation kind vs the pattern's ceiling: every run a fresh process (fresh allocations)
set -o pipefail
TAG=${1:-r05t}
mkdir -p gpurun_out
P=./tools/depth_probe
run() { timeout -k 5 60 $P "$@" | tee -a gpurun_out/${TAG}_alloc.log || exit 1; }
for rep in 1 2 3 4; do
  for lay in 0 2 3; do
    run 10000 5451 18 12 20 1 2 0 0 $lay
    run 1250 5451 54 12 20 1 2 0 0 $lay
  done
done
