#!/bin/bash
# Round 5, lease d: one-lease shard table (10 k cells vs the 8/4/2-GPU per-rank shards with the
# library's RCCL all-reduce at world 1), the C1 fresh-process full fit, the C4 full fit.
set -o pipefail
TAG=${1:-r05d}
mkdir -p gpurun_out
rm -f gpurun_out/${TAG}_shards.jsonl
for rep in 1 2; do
  for cfg in "--cells 10000" "--cells 1250 --comm rccl" "--cells 1250 --comm rccl --fused" "--cells 2500 --comm rccl" \
             "--cells 5000 --comm rccl"; do
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $cfg > gpurun_out/${TAG}_bench.tmp 2>&1 \
      || { cat gpurun_out/${TAG}_bench.tmp; exit 1; }
    grep '"metric"' gpurun_out/${TAG}_bench.tmp | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_fused']=('--fused' in '$cfg')
print(json.dumps(r))" >> gpurun_out/${TAG}_shards.jsonl
    echo "rep $rep: $cfg done"
  done
done
python tools/shard_table.py gpurun_out/${TAG}_shards.jsonl | tee gpurun_out/${TAG}_shard_sizes.log
timeout -k 10 200 python -u bench.py --fullfit-c1 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err \
  || { tail -20 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/${TAG}_fullfit_c1.json')); print('C1 gpu %.3f s (import %.3f s) cpu %.2f s speedup %.1f' % (r['gpu_s'], r['gpu_import_s'], r['cpu_baseline']['seconds'], r['speedup']))"
timeout -k 10 300 python -u tools/fullfit_bench.py --config c4 --n-jobs 1 --cpu-sample-cells 0 \
  > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -20 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
python -c "
import json; r=json.load(open('gpurun_out/${TAG}_fullfit_c4.json')); t=r['timings_s']; print('C4 total %.2f s' % t['total'], t['phases'], r['iters'], r['ms_per_step'])"
