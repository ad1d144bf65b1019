#!/bin/bash
# Full-fit wall clock of the drop-in pipeline at C3 and C4 with the
# CPU-oracle extrapolation; one JSON line per config under gpurun_out/.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
for c in c3 c4; do
  timeout -k 10 900 python -u tools/fullfit_bench.py --config $c > gpurun_out/${TAG}_fullfit_$c.json 2> gpurun_out/${TAG}_fullfit_$c.err || { tail -20 gpurun_out/${TAG}_fullfit_$c.err; exit 1; }
  tail -c 600 gpurun_out/${TAG}_fullfit_$c.json
done
