#!/bin/bash
# Standard GPU round (repo root on the box): the -m gpu parity suite, the default bench
# (with cpu_baseline) and the strong-scaling per-rank shard sizes of configs[3] on one GPU.
# usage: tools/gpu_check.sh TAG [--quick]
set -o pipefail
TAG=${1:-run}; shift || true
mkdir -p gpurun_out
# PYTEST_K: an optional -k expression (e.g. to leave out a test under rework)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
if [ "$1" != "--quick" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log
fi
for c in 1250 2500 5000; do
  timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --cells $c > gpurun_out/${TAG}_cells$c.log 2>&1 || exit 1
  python -c "
import json; r=json.loads(open('gpurun_out/${TAG}_cells$c.log').read().strip().splitlines()[-1]); print('cells $c', round(r['ms_per_step'],4), round(r['roofline']['kernel_ms'],4), r['config'].get('bins_per_tile'))"
done
