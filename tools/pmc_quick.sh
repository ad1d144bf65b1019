#!/bin/bash
# Two SQ counter passes (instruction mix, busy/wait cycles) of the enumerated pass for one
# bench configuration; prints per-launch means.  usage: tools/pmc_quick.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/pmcq_$TAG
mkdir -p "$OUT"
ARGS=${*:-"--steps 5 --warmup 1 --no-cpu-baseline"}
cd /tmp && export TMPDIR=/tmp
K="--kernel-include-regex ${KREGEX:-enum_dma}"
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC $K -d "$OUT/pmc$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/pmc$i.log" 2>&1
done
cd "$R" && python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for cs in per.values():
        for c, v in cs.items():
            acc[c].append(v)
for k, v in sorted(acc.items()):
    print("{:28s} {:.4g}".format(k, sum(v) / max(1, len(v))))
PY
