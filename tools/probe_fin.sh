#!/bin/bash
# finalize attribution. ab/probe.so = a build of pert_kernels.hip whose pert_finalize reads
# PERT_FIN_PROBE (not kept in-tree): 1 = an empty kernel before
# finalize, 2 = + only the per-bin blocks, 3 = + only the per-cell blocks
set -o pipefail
R=$(pwd)
export PERT_LIB=$R/ab/probe.so
cd /tmp && export TMPDIR=/tmp
for m in 1 2 3; do
  for c in 1250 10000; do
    D=$R/gpurun_out/probe_${m}_$c
    mkdir -p $D
    PERT_FIN_PROBE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --cells $c --steps 20 > $D/log.txt 2>&1 || exit 1
    f=$(find $D -name '*kernel_trace.csv' | head -1)
    echo "== probe $m cells $c"; python3 $R/tools/trace_steps.py $f
  done
done
