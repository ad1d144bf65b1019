#!/bin/bash
# Kernel-trace A/B (rocprofv3 --kernel-trace --stats) of this tree's library against a variant
# build:   bash tools/trace_ab.sh TAG VARIANT.so [bench args...]
set -eo pipefail
TAG=$1; VAR=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for which in tree variant; do
  if [ "$which" = variant ]; then export PERT_LIB=$R/$VAR; else unset PERT_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$which" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/trace_$which.log" 2>&1
done
