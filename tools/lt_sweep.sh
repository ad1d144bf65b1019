#!/bin/bash
# bins-per-tile sweep: "CELLS LT" pairs from the command line (LT 0 = auto)
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  set -- ${spec/:/ }
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --cells $1 --bins-per-tile $2 > gpurun_out/sw_$1_$2.log 2>&1 || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/sw_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', round(r['ms_per_step'],4), round(r['roofline']['kernel_ms'],4), r['config'].get('bins_per_tile'))"
done
