#!/bin/bash
# Round-4 performance lease: pass-timing events on/off (C4, the 1,250-cell shard, step 1), a
# kernel trace of the step-1 bench (launch gaps), the C5 pass's VALU count (PMC), and the C4
# and C1 full fits at HEAD.
set -o pipefail
TAG=${1:-r04i}
mkdir -p gpurun_out
O=gpurun_out/${TAG}_events.log; : > $O
row() {
  local label=$1; shift
  timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  python -c "
import json; r=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); rf=r['roofline']
print('$label', 'cells', r['config']['cells'], 'fit', r['config']['fit'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'],4), 'pass_ms', round(rf['kernel_ms'],4), 'ceiling', round(rf.get('pattern_ceiling', {}).get('ms', 0),4))" | tee -a $O
}
for es in 1 10 0; do
  row "c4 es$es" --event-stride $es || exit 1
  row "shard es$es" --cells 1250 --event-stride $es || exit 1
  row "step1 es$es" --fit step1 --event-stride $es || exit 1
done
row "shard fused es0" --cells 1250 --event-stride 0 --fused || exit 1
R=$(pwd)
mkdir -p gpurun_out/prof_${TAG}_s1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_s1/trace -o run --output-format csv -- python3 $R/bench.py --fit step1 --steps 20 --warmup 3 --no-cpu-baseline --event-stride 0 > $R/gpurun_out/prof_${TAG}_s1/trace.log 2>&1) || { tail -5 gpurun_out/prof_${TAG}_s1/trace.log; exit 1; }
mkdir -p gpurun_out/prof_${TAG}_c5
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS --kernel-include-regex 'enum3_' -d $R/gpurun_out/prof_${TAG}_c5/pmc1 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_${TAG}_c5/pmc1.log 2>&1) || { tail -5 gpurun_out/prof_${TAG}_c5/pmc1.log; exit 1; }
timeout -k 10 300 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -5 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/${TAG}_fullfit_c4.json').read().strip().splitlines()[-1])
t=d['timings_s']; print(t['phases']); print('ms_per_step', d['ms_per_step'], 'total', t['total'])"
timeout -k 10 200 python -u tools/fullfit_bench.py --config c1 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err || { tail -5 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
tail -c 600 gpurun_out/${TAG}_fullfit_c1.json
