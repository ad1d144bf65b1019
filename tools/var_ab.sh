#!/bin/bash
# A/B of enumerated-pass variants / tile lengths in one box, interleaved, 3 rounds:
#   tools/var_ab.sh "0 3 3:32" "1250 10000"     (variant[:bins_per_tile])
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for c in $2; do for vs in $1; do
 v=${vs%%:*}; lt=0; [[ $vs == *:* ]] && lt=${vs##*:}
 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c --variant $v --bins-per-tile $lt > gpurun_out/var_${c}_${v}_$lt.log 2>&1 || exit 1
 python -c "
import json; r=json.loads(open('gpurun_out/var_${c}_${v}_$lt.log').read().strip().splitlines()[-1]); print('$r cells $c var $vs LT', r['config']['bins_per_tile'], round(r['ms_per_step'],4), round(r['roofline']['kernel_ms'],4))"
done; done; done
