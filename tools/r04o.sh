#!/bin/bash
# GPU suite after the finalize / planner changes, then the A/B against the previous commit's build.
set -o pipefail
TAG=${1:-r04o}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_chain.py::test_genome_length_chain_matches_oracle_fixture > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
bash tools/ab_bench.sh ${TAG} ab/libpert_head.so || exit 1
