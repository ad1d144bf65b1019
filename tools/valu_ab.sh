#!/bin/bash
# VALU instructions of the enumerated pass, this tree's library against a variant build, one
# --pmc pass each (rocprofv3; counters only, no other tracing):
#   bash tools/valu_ab.sh TAG VARIANT.so [bench args...]
set -eo pipefail
TAG=$1; VAR=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export PERT_PLACEMENT=0
for which in tree variant; do
  if [ "$which" = variant ]; then export PERT_LIB=$R/$VAR; else unset PERT_LIB; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES --kernel-include-regex 'enum3_kernel' \
    --output-format csv -d "$OUT/valu_$which" -o run -- python3 "$R/bench.py" --no-cpu-baseline --steps 4 --warmup 1 "$@" \
    > "$OUT/valu_$which.log" 2>&1
done
