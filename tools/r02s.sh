#!/bin/bash
# round-2 evidence on one lease: GPU tests, smoke, rocprof trace + PMC of the default bench,
# then the default bench reading that profile (roofline frac from the trace, traffic from PMC)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02s_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s_smoke.log 2>&1 || exit $?
timeout -k 10 1000 bash tools/profile.sh r02s || exit $?
python3 tools/pmc_traffic.py gpurun_out/prof_r02s/summary.json c4 10000 profiles/pmc_traffic.json || exit $?
cp profiles/pmc_traffic.json gpurun_out/r02s_pmc_traffic.json
timeout -k 10 400 python bench.py --profile gpurun_out/prof_r02s > gpurun_out/r02s_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r02s_bench_default.log
