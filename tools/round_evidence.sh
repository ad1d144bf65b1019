#!/bin/bash
# One round's evidence on the GPU box (repo root): the -m gpu suite, smoke(), the default bench
# (with cpu_baseline), the per-rank shard sizes of configs[3], rocprofv3 trace + PMC of the bench,
# the step-1 bench, and the C1 / C4 full fits.  Every step under its own time limit; the first
# failure ends the script.
# usage: tools/round_evidence.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 1000 bash tools/profile.sh $TAG || exit 1
bash tools/fit_evidence.sh $TAG --no-profile || exit 1
