#!/bin/bash
# A/B libpert_hip builds on one box for each fit kind: tools/ab_fit.sh "libA.so libB.so" "step1 step2" [bench args]
set -o pipefail
LIBS=$1; FITS=$2; shift 2
ARGS=${*:-"--no-cpu-baseline"}
mkdir -p gpurun_out
for round in 1 2; do for F in $FITS; do for L in $LIBS; do
  PERT_LIB=$(pwd)/scdna_replication_tools_amd/$L timeout -k 10 200 python bench.py --fit $F $ARGS > gpurun_out/abf_${L}_${F}_$round.log 2>&1 || { tail -5 gpurun_out/abf_${L}_${F}_$round.log; exit 1; }
  echo "$round $F $L $(tail -1 gpurun_out/abf_${L}_${F}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "frac", round(d["roofline"]["frac"],3))')"
done; done; done
