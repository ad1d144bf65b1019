#!/bin/bash
# Round 5, first lease: the GPU suite at HEAD, then the loader probe of a two-rank fit.
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Timeout" gpurun_out/${TAG}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/dl_probe.py --world2 > gpurun_out/${TAG}_dlprobe.log 2>&1; rc2=$?
tail -40 gpurun_out/${TAG}_dlprobe.log
exit $(( rc > rc2 ? rc : rc2 ))
