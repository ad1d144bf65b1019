#!/bin/bash
# The sharded step's all-reduce overlap: the 1,250-cell shard (N = 8 of C4)
# and the 10 k step at world 1, with the split step (overlap 1) or the sequential one (0), with
# and without a 20 us stand-in kernel in every all-reduce (an 8-rank ring's latency), interleaved.
#   bash tools/overlap_ab.sh TAG [REPS] [extra bench args...]
set -eo pipefail
TAG=$1; REPS=${2:-2}; shift; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rm -f "$OUT/overlap.jsonl"
run() {
  local rep=$1; shift
  timeout -k 10 240 python -u bench.py --steps 200 --warmup 3 --no-cpu-baseline "$@" > "$OUT/b.tmp" 2>&1 \
    || { cat "$OUT/b.tmp"; exit 1; }
  grep '"metric"' "$OUT/b.tmp" | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_rep']=$rep; r['_args']='$*'
print(json.dumps(r))" >> "$OUT/overlap.jsonl"
  python -c "import json; r=[json.loads(l) for l in open('$OUT/overlap.jsonl')][-1]; print('rep $rep $*: %.4f ms/step (evented %.4f), pass %.4f' % (r['ms_per_step'], r['ms_per_step_evented'], r['roofline']['kernel_ms']))"
}
for rep in $(seq 1 "$REPS"); do
  run "$rep" --cells 10000 "$@"
  for d in 0 20; do
    for o in 0 1; do
      run "$rep" --cells 1250 --comm rccl --comm-overlap $o --comm-delay-us $d "$@"
    done
  done
  run "$rep" --cells 2500 --comm rccl --comm-overlap 1 "$@"
  run "$rep" --cells 5000 --comm rccl --comm-overlap 1 "$@"
done
