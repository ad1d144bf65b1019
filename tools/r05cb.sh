#!/bin/bash
# Round 5, lease cb: the shard table at K = 200 (the bench default), with the placement search
# library's RCCL all-reduce at world 1), then the C4 full fit end to end.
set -o pipefail
TAG=${1:-r05cb}
mkdir -p gpurun_out
rm -f gpurun_out/${TAG}_shards.jsonl
run() {
  local rep=$1; shift
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${TAG}_b.tmp 2>&1 \
    || { cat gpurun_out/${TAG}_b.tmp; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_b.tmp | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_fused']=False
print(json.dumps(r))" >> gpurun_out/${TAG}_shards.jsonl
  echo "rep $rep $*: $(python -c "import json; r=[json.loads(l) for l in open('gpurun_out/${TAG}_shards.jsonl')][-1]; print(r['ms_per_step'], r['roofline'].get('pi_placement',{}).get('candidates_ms'))")"
}
for rep in 1 2; do
  run $rep --cells 10000
  run $rep --cells 1250 --comm rccl
  run $rep --cells 2500 --comm rccl
  run $rep --cells 5000 --comm rccl
  run $rep --config c5
  run $rep --config c5 --cells 250 --comm rccl
done
python tools/shard_table.py gpurun_out/${TAG}_shards.jsonl | tee gpurun_out/${TAG}_shard_sizes.log
