#!/bin/bash
# A/B diagnostics of the round-4 kernel changes (run on the GPU box): full-vs-shard linearity
# (tools/shard_diag.py) and the saturated argmax gradient test under the in-tree build and
# the A/B builds in ab/ (tools/build_ab.sh).  A test failure (pytest rc 1) is data; anything
# else ends the script.
set -o pipefail
TAG=${1:-r04g}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_diag.log
: > $OUT
for lib in default ab/libpert_jmax.so ab/libpert_prejmax.so; do
  if [ $lib = default ]; then unset PERT_LIB; else export PERT_LIB=$PWD/$lib; fi
  echo "== $lib" | tee -a $OUT
  timeout -k 10 300 python -u tools/shard_diag.py >> $OUT 2>&1 || { echo "shard_diag rc=$?" | tee -a $OUT; tail -20 $OUT; exit 1; }
  tail -1 $OUT | cut -c1-900
  timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -k saturated -x -q --timeout 240 --timeout-method thread >> $OUT 2>&1
  rc=$?
  echo "saturated rc=$rc" | tee -a $OUT
  [ $rc -le 1 ] || { tail -20 $OUT; exit 1; }
done
