#!/bin/bash
# Interleaved A/B of two bench flag sets on one lease:
#   bash tools/flag_ab.sh TAG REPS "FLAGS_A" "FLAGS_B" [common bench args...]
set -eo pipefail
TAG=$1; REPS=$2; A=$3; B=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for f in "$A" "$B"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $f "$@" > "$OUT/b.tmp" 2>&1 || { cat "$OUT/b.tmp"; exit 1; }
    grep '"metric"' "$OUT/b.tmp" >> "$OUT/flags.jsonl"
    python -c "import json; r=[json.loads(l) for l in open('$OUT/flags.jsonl')][-1]; rf=r['roofline']; print('%-30s: %.4f ms/step, pass %.4f ms, ceiling %.4f' % ('$f', r['ms_per_step'], rf['kernel_ms'], rf['pattern_ceiling']['ms']))"
  done
done
