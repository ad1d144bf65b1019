#!/bin/bash
# Round-4 closing evidence from one lease at HEAD: smoke, the default bench line, roofline
# evidence (trace + PMC + bench --profile), per-rank shard sizes, step 1, the two-rank bench path
# (gloo, one GPU), and the C4 / C1 full fits.
set -o pipefail
TAG=${1:-r04z}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_default.log | cut -c1-400
bash tools/roofline_evidence.sh $TAG || exit 1
O=gpurun_out/${TAG}_shard_sizes.log; : > $O
for c in 10000 5000 2500 1250; do
  timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --cells $c > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  python -c "
import json; r=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); rf=r['roofline']
print('cells', r['config']['cells'], 'LT', r['config']['bins_per_tile'], 'step_ms', round(r['ms_per_step'],4), 'pass_ms', round(rf['kernel_ms'],4), 'ceiling', round(rf['pattern_ceiling']['ms'],4))" | tee -a $O
done
timeout -k 10 150 python bench.py --fit step1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_step1.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_step1.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_step1.log | cut -c1-300
PERT_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_gloo2.log 2>&1 || { tail -20 gpurun_out/${TAG}_gloo2.log; exit 1; }
grep '^{' gpurun_out/${TAG}_gloo2.log | tail -1 | cut -c1-300
timeout -k 10 300 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -5 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/${TAG}_fullfit_c4.json').read().strip().splitlines()[-1])
t=d['timings_s']; print(t['phases']); print('ms_per_step', d['ms_per_step'], 'iters', d['iters'], 'total', t['total'])"
timeout -k 10 200 python -u tools/fullfit_bench.py --config c1 --cpu-sample-cells 0 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err || { tail -5 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
tail -c 300 gpurun_out/${TAG}_fullfit_c1.json
