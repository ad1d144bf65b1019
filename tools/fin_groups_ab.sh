#!/bin/bash
# finalize's bin-tile groups (PERT_FIN_GROUPS) under a kernel trace:
#   bash tools/fin_groups_ab.sh TAG "G1 G2 ..." [bench args...]      (G = 1: one workgroup per 64 cells)
set -eo pipefail
TAG=$1; GS=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for g in $GS; do
  export PERT_FIN_GROUPS=$g
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g$g" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/g$g.log" 2>&1
  echo "groups $g: $(grep -h 'finalize_kernel' $OUT/g$g/run_kernel_stats.csv | awk -F',' '{print $(NF-4)}') ns finalize; $(grep -h '"metric"' $OUT/g$g.log | python3 -c 'import json,sys; r=json.load(sys.stdin); print(round(r["ms_per_step"],4), "ms/step")')"
done
