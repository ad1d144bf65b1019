#!/bin/bash
# Round-4 lease after the enum3 LDS-DMA wait fix: step 2 alone from the fixture's step-1 sites
# (tools/gpu_step2_probe.py), the genome chain (product dump incl. its step-1 beta_means), the
# whole -m gpu suite, the full-vs-shard linearity diagnostic and the default bench.
set -o pipefail
TAG=${1:-r04h}
mkdir -p gpurun_out
export PERT_DUMP_DIR=gpurun_out
timeout -k 10 400 python -u tools/gpu_step2_probe.py --out gpurun_out/${TAG}_step2_probe.npz > gpurun_out/${TAG}_step2_probe.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_step2_probe.log; exit 1; }
tail -1 gpurun_out/${TAG}_step2_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -k genome \
  > gpurun_out/${TAG}_genome.log 2>&1; rc=$?
grep -E "genome chain vs oracle|PASS|FAIL|Error" gpurun_out/${TAG}_genome.log | cut -c1-1500 | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_chain.py::test_genome_length_chain_matches_oracle_fixture \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u tools/shard_diag.py > gpurun_out/${TAG}_shard_diag.log 2>&1 || { tail -5 gpurun_out/${TAG}_shard_diag.log; exit 1; }
tail -1 gpurun_out/${TAG}_shard_diag.log | cut -c1-600
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
