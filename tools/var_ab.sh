#!/bin/bash
# A/B of enumerated-pass variants in one box: tools/var_ab.sh "0 2" "1250 10000"
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for c in $2; do for v in $1; do
 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c --variant $v > gpurun_out/var_${c}_$v.log 2>&1 || exit 1
 python -c "
import json; r=json.loads(open('gpurun_out/var_${c}_$v.log').read().strip().splitlines()[-1]); print('$r cells $c var $v', round(r['ms_per_step'],4), round(r['roofline']['kernel_ms'],4))"
done; done; done
