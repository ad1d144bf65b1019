#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_chain.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r02k_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/r02k_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
for r in 1 2; do
for c in 10000 1250; do
for a in "v0on --variant 0" "v0fw --variant 0" "v0on --variant 3 --no-fused"; do
  set -- $a; lib=$1; shift
  PERT_LIB=$(pwd)/scdna_replication_tools_amd/ab_$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c "$@" > gpurun_out/r02k_b.log 2>&1 || exit $?
  echo "$r $c $a $(tail -1 gpurun_out/r02k_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02k_ab.log
done
done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lib in v0on v0fw; do
  PERT_LIB=$R/scdna_replication_tools_amd/ab_$lib.so timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex enum_ -d $R/gpurun_out/pmck_$lib -o run --output-format csv -- python3 $R/bench.py --variant 0 --steps 4 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmck_$lib.log 2>&1 || exit $?
done
