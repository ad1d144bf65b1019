#!/bin/bash
# Runs only on a "fast" box (the 10 k pattern ceiling below 3.1 ms: HBM at ~6 TB/s for the large
# launch): what holds the per-rank shards' ceiling there -- tile length and launch size of the
# pattern (depth_probe), and the 1,250 / 2,500-cell steps at other tile lengths vs the 10 k step.
set -o pipefail
TAG=${1:-fast}
mkdir -p gpurun_out
line=$(timeout -k 5 60 ./tools/depth_probe 10000 5451 18 12 20 1 2) || exit 1
echo "$line" | tee -a gpurun_out/${TAG}_fastbox.log
ms=$(echo "$line" | sed -E 's/.*depth1 ([0-9.]+) ms.*/\1/')
if python -c "import sys; sys.exit(0 if float('$ms') < 3.1 else 1)"; then
  echo "fast box ($ms ms): sweep" | tee -a gpurun_out/${TAG}_fastbox.log
  for args in "10000 5451 12 12" "10000 5451 54 12" "5000 5451 12 12" "5000 5451 18 12" "5000 5451 36 12" \
              "2500 5451 12 12" "2500 5451 18 12" "2500 5451 27 12" "1250 5451 18 12" "1250 5451 27 12" \
              "1250 5451 54 12" "1250 5451 54 8" "20000 5451 18 12"; do
    timeout -k 5 60 ./tools/depth_probe $args 20 1 2 | tee -a gpurun_out/${TAG}_fastbox.log || exit 1
  done
  for args in "10000 5451 54 12 20 1 2 0 20" "10000 5451 18 12 20 1 2 0 20" "10000 5451 18 12 20 1 2 0 80" \
              "1250 5451 54 12 20 8 2" "1250 5451 6 12 20 1 2"; do
    timeout -k 5 60 ./tools/depth_probe $args | tee -a gpurun_out/${TAG}_fastbox.log || exit 1
  done
  for w in 256 512 1024; do
    for args in "1250 5451 54 12" "10000 5451 18 12"; do
      timeout -k 5 60 ./tools/depth_probe $args 20 1 2 $w | tee -a gpurun_out/${TAG}_fastbox.log || exit 1
    done
  done
else
  echo "slow box ($ms ms): no sweep" | tee -a gpurun_out/${TAG}_fastbox.log
  timeout -k 5 60 ./tools/depth_probe 10000 5451 54 12 20 1 2 0 20 | tee -a gpurun_out/${TAG}_fastbox.log || exit 1
fi
