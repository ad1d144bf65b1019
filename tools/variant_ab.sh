#!/bin/bash
# In-lease A/B of this tree's library against a variant build (tools/build_variant_lib.sh),
# interleaved:   bash tools/variant_ab.sh TAG VARIANT.so REPS [bench args...]
set -eo pipefail
TAG=$1; VAR=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
  local which=$1; shift
  if [ "$which" = variant ]; then export PERT_LIB=$VAR; else unset PERT_LIB; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/b.tmp" 2>&1 || { cat "$OUT/b.tmp"; exit 1; }
  grep '"metric"' "$OUT/b.tmp" | python -c "
import json,sys
r=json.loads(sys.stdin.read()); r['_which']='$which'; r['_args']='$*'
print(json.dumps(r))" >> "$OUT/ab.jsonl"
  python -c "import json; r=[json.loads(l) for l in open('$OUT/ab.jsonl')][-1]; rf=r['roofline']; print('%-8s $*: %.4f ms/step, pass %.4f ms, ceiling %s' % ('$which', r['ms_per_step'], rf['kernel_ms'], rf.get('pattern_ceiling',{}).get('ms')))"
}
for rep in $(seq 1 "$REPS"); do
  run tree "$@"
  run variant "$@"
done
