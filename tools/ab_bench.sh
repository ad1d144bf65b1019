#!/bin/bash
# A/B the enumerated pass across libpert_hip builds on one box (interleaved, 2 rounds).
#   tools/ab_bench.sh "libA.so libB.so ..." [bench args]
set -o pipefail
LIBS=$1; shift
ARGS=${*:-"--no-cpu-baseline"}
mkdir -p gpurun_out
for round in 1 2; do
  for L in $LIBS; do
    PERT_LIB=$(pwd)/scdna_replication_tools_amd/$L timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab_${L}_$round.log 2>&1 || exit 1
    echo "$round $L $(tail -1 gpurun_out/ab_${L}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4))')"
  done
done
