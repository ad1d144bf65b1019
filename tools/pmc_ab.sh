#!/bin/bash
# Two SQ PMC passes (counters as tools/profile.sh) of the bench for each variant given:
#   tools/pmc_ab.sh "0 3" [extra bench args]
# Results: gpurun_out/pmcab_v<variant>_<pass>/ ; summary printed by tools/pmc_summary.py.
R=$(pwd)
VARS=$1; shift
ARGS=${*:-"--steps 4 --warmup 1 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
K='--kernel-include-regex enum_|enum3_'
for v in $VARS; do
  OUT=$R/gpurun_out/pmcab_v$v
  mkdir -p "$OUT"
  i=0
  for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $PMC $K -d "$OUT/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" --variant $v $ARGS > "$OUT/pmc$i.log" 2>&1 || exit $?
  done
  (cd "$R" && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json")
done
