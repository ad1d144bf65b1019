#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_bench.sh "ab_g6w3.so ab_gmem.so ab_fwdw2.so ab_fwdgmw2.so" --no-cpu-baseline --variant 3 --steps 20 --warmup 3 > gpurun_out/r02g_ab.log 2>&1 || exit $?
PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_g6w3.so timeout -k 10 200 python bench.py --no-cpu-baseline --variant 3 --no-fused --steps 20 --warmup 3 > gpurun_out/r02g_nofused.log 2>&1 || exit $?
PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_g6w3.so timeout -k 10 200 python bench.py --no-cpu-baseline --variant 0 --steps 20 --warmup 3 > gpurun_out/r02g_v0.log 2>&1
