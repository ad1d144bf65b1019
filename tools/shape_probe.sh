#!/bin/bash
# Per-cell.bin cost of the enumerated pass vs shard shape at constant coverage (reads per bin):
# cells x (5451 x sub) bins with sub x 1e6 reads per cell.
set -o pipefail
mkdir -p gpurun_out
for spec in "10000 1" "1250 1" "1250 8" "2500 4" "5000 2" "10000 1"; do set -- $spec
 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --cells $1 --subdivide $2 --reads-per-cell ${2}e6 > gpurun_out/shape_$1_$2.log 2>&1 || exit 1
 python -c "
import json; r=json.loads(open('gpurun_out/shape_$1_$2.log').read().strip().splitlines()[-1]); c=r['config']; print('cells $1 sub $2 LT', c['bins_per_tile'], 'kernel', round(r['roofline']['kernel_ms'],4), 'ps/cb', round(r['roofline']['kernel_ms']*1e9/(c['cells']*c['bins']),2))"
done
