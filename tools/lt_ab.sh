#!/bin/bash
# Tile-length A/B on one lease: bash tools/lt_ab.sh TAG "LT1 LT2 ..." REPS [bench args...]
set -eo pipefail
TAG=$1; LTS=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 "$REPS"); do
  for lt in $LTS; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --bins-per-tile $lt "$@" > "$OUT/b.tmp" 2>&1 || { cat "$OUT/b.tmp"; exit 1; }
    grep '"metric"' "$OUT/b.tmp" >> "$OUT/lt.jsonl"
    python -c "import json; r=[json.loads(l) for l in open('$OUT/lt.jsonl')][-1]; rf=r['roofline']; print('LT %3d $*: %.4f ms/step, pass %.4f ms, ceiling %.4f' % (r['config']['bins_per_tile'], r['ms_per_step'], rf['kernel_ms'], rf['pattern_ceiling']['ms']))"
  done
done
