#!/bin/bash
# Counter passes of tools/placement_probe.py (one --pmc run per pass, counters only), then
# tools/placement_pmc.py:   bash tools/placement_pmc.sh TAG
set -eo pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
K="--kernel-include-regex stream_ceiling"
i=0
for PMC in "TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum" \
           "TCC_EA0_WRREQ TCC_EA0_RDREQ" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $PMC $K --output-format csv -d "$OUT/pmc$i" -o run -- \
    python3 "$R/tools/placement_probe.py" > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.log"
done
cd "$R" && python3 tools/placement_pmc.py "$OUT" > "$OUT/summary.json"
