#!/bin/bash
# the default bench (K = 200) under rocprofv3 --kernel-trace --stats: enum3_kernel's average against the line's kernel_ms
set -o pipefail
mkdir -p gpurun_out/r05cd_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05cd_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/r05cd_prof/bench.log 2>&1
