#!/bin/bash
# The one-lease strong-scaling table: the 10 k-cell C4 step and the
# per-rank shards of N = 2/4/8 (and C5's 250-cell shard) with the library's all-reduce at world 1,
# each a bench.py run appended to gpurun_out/TAG/shards.jsonl, then tools/shard_table.py.
#   bash tools/shard_runs.sh TAG [REPS] [extra bench args...]
set -eo pipefail
TAG=$1; REPS=${2:-2}; shift; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rm -f "$OUT/shards.jsonl"
run() {
  local rep=$1; shift
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 3 --no-cpu-baseline "$@" > "$OUT/b.tmp" 2>&1 \
    || { cat "$OUT/b.tmp"; exit 1; }
  grep '"metric"' "$OUT/b.tmp" | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_fused']=False
print(json.dumps(r))" >> "$OUT/shards.jsonl"
  echo "rep $rep $*: $(python -c "import json; r=[json.loads(l) for l in open('$OUT/shards.jsonl')][-1]; print(r['ms_per_step'])")"
}
for rep in $(seq 1 "$REPS"); do
  run "$rep" --cells 10000 "$@"
  run "$rep" --cells 1250 --comm rccl "$@"
  run "$rep" --cells 2500 --comm rccl "$@"
  run "$rep" --cells 5000 --comm rccl "$@"
  run "$rep" --config c5 "$@"
  run "$rep" --config c5 --cells 250 --comm rccl "$@"
done
python tools/shard_table.py "$OUT/shards.jsonl" | tee "$OUT/shard_sizes.log"
