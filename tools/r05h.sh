#!/bin/bash
# Round 5, lease h: the bench with the pattern-ceiling warm-up before the timed region; shard
# tables of C4 (10 k cells vs the 2/4/8-GPU shards) and C5 (2,000 cells x 136,275 bins vs the
# 8-GPU shard of 250 cells), the library's RCCL all-reduce at world 1.
set -o pipefail
TAG=${1:-r05h}
mkdir -p gpurun_out
rm -f gpurun_out/${TAG}_shards.jsonl
run() {
  local rep=$1; shift
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/${TAG}_b.tmp 2>&1 \
    || { cat gpurun_out/${TAG}_b.tmp; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_b.tmp | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_fused']=False
print(json.dumps(r))" >> gpurun_out/${TAG}_shards.jsonl
  echo "rep $rep $*: done"
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
