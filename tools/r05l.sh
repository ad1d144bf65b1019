#!/bin/bash
# the load-schedule experiment (depth_probe work mode, constant-index arithmetic), then the
# fast-box sweep when the box is fast
set -o pipefail
TAG=${1:-r05l}
mkdir -p gpurun_out
for w in 0 256 512 1024 2048; do
  for args in "1250 5451 54 12" "10000 5451 18 12"; do
    if [ $w -eq 0 ]; then timeout -k 5 60 ./tools/depth_probe $args 20 1 2 | tee -a gpurun_out/${TAG}_work.log || exit 1
    else timeout -k 5 60 ./tools/depth_probe $args 20 1 2 $w | tee -a gpurun_out/${TAG}_work.log || exit 1; fi
  done
done
bash tools/fastbox_sweep.sh ${TAG}
