#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_bench.sh "ab_g6w3.so ab_g18w2.so ab_g9w3.so ab_g6w2.so" --no-cpu-baseline --variant 3 --steps 20 --warmup 3 > gpurun_out/r02f_ab.log 2>&1 || exit $?
PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_g6w3.so timeout -k 10 200 python bench.py --no-cpu-baseline --variant 0 --steps 20 --warmup 3 > gpurun_out/r02f_v0.log 2>&1
