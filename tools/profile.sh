#!/bin/bash
# rocprofv3 evidence for the dominant kernel (run on the GPU box from the repo root):
#   kernel-trace stats of the bench, then separate --pmc passes (never combined with
#   other tracing), parsed into profiles/ by tools/pmc_summary.py.
# usage: tools/profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--steps 10 --warmup 2 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
K='--kernel-include-regex enum_|enum3_|obs_|finalize_kernel|adam_kernel'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC $K -d "$OUT/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc$i.log" 2>&1
done
cd "$R" && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json"
