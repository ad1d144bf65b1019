#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for spec in "1250 16" "1250 18" "1250 9" "1250 12" "1250 32" "10000 64" "10000 54" "10000 62" "10000 48"; do
  set -- $spec
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --cells $1 --bins-per-tile $2 > gpurun_out/sw_$1_$2.log 2>&1 || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/sw_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', round(r['ms_per_step'],4), round(r['roofline']['kernel_ms'],4))"
done
