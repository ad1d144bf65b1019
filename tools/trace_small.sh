#!/bin/bash
# kernel traces of a small shard (the per-rank work of an 8-GPU strong-scaling run of
# configs[3]) and of the default bench; per-step timelines by tools/trace_steps.py
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/trace_small gpurun_out/trace_c4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_small -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --cells 1250 --steps 30 > $R/gpurun_out/trace_small/log.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace_c4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 > $R/gpurun_out/trace_c4/log.txt 2>&1 || exit 1
cd $R
for d in trace_small trace_c4; do
  f=$(find gpurun_out/$d -name '*kernel_trace.csv' | head -1)
  echo "== $d"; python3 tools/trace_steps.py $f
done
