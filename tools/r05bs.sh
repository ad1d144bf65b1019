#!/bin/bash
# Round 5, lease bs: at HEAD -- GPU suite, smoke, the default bench line, then the default bench
# under rocprofv3 --kernel-trace --stats (its enum3_kernel average against the bench's HIP-event figure).
set -o pipefail
TAG=${1:-r05bs}
bash tools/r05bk.sh $TAG || exit $?
mkdir -p gpurun_out/${TAG}_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/bench.log 2>&1
