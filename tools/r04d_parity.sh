#!/bin/bash
# Parity evidence after the argmax-logit gradient change: the genome-length chain (product dump
# kept for offline analysis), then the whole -m gpu suite and the default bench.
set -o pipefail
mkdir -p gpurun_out
export PERT_DUMP_DIR=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -k genome \
  > gpurun_out/r04d_genome.log 2>&1; rc=$?
grep -E "genome chain vs oracle|PASS|FAIL|Error" gpurun_out/r04d_genome.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_chain.py::test_genome_length_chain_matches_oracle_fixture \
  > gpurun_out/r04d_tests.log 2>&1 || { tail -30 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r04d_bench.log 2>&1 || { tail -20 gpurun_out/r04d_bench.log; exit 1; }
tail -1 gpurun_out/r04d_bench.log | cut -c1-700
