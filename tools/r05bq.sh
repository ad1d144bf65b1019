#!/bin/bash
# kernel trace of the 1,250-cell sharded step (RCCL at world 1): per-kernel durations and the gaps
set -o pipefail
mkdir -p gpurun_out/r05bq
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05bq -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --cells 1250 --comm rccl --steps 200 > $GRAFT_REPO_ROOT/gpurun_out/r05bq/bench.log 2>&1
