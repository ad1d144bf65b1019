#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02ad_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/r02ad_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02ad_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r02ad_smoke.log
