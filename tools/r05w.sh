#!/bin/bash
# wave timeline of the three-wave pass (stamps build) at 1,250 cells (LT 54, 27) and 10 k (LT 18)
set -o pipefail
mkdir -p gpurun_out
for c in "1250 54" "1250 27" "10000 18"; do
  set -- $c
  echo "== cells $1 LT $2" >> gpurun_out/r05w_timeline.log
  PERT_LIB=tools/_stamps.so VARIANT=3 LT=$2 timeout -k 10 120 python tools/wave_timeline.py $1 >> gpurun_out/r05w_timeline.log 2>&1 || exit 1
done
cat gpurun_out/r05w_timeline.log
