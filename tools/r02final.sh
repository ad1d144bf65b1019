#!/bin/bash
# round-2 final evidence on one lease: GPU suite, smoke, rocprof trace + PMC of the default
# bench, the default bench reading that profile, and the bench's N>1 path rehearsed with two
# gloo ranks on the one GPU
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02f_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02f_smoke.log 2>&1 || exit $?
timeout -k 10 1000 bash tools/profile.sh r02f || exit $?
python3 tools/pmc_traffic.py gpurun_out/prof_r02f/summary.json c4 10000 profiles/pmc_traffic.json || exit $?
cp profiles/pmc_traffic.json gpurun_out/r02f_pmc_traffic.json
timeout -k 10 400 python bench.py --profile gpurun_out/prof_r02f > gpurun_out/r02f_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r02f_bench_default.log
PERT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/r02f_gloo2.log 2>&1 || exit $?
tail -1 gpurun_out/r02f_gloo2.log
