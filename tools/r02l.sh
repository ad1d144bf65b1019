#!/bin/bash
# round-2 re-entry check: full GPU suite, smoke, default bench, variant-0 vs variant-3 A/B
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02l_tests.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/r02l_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02l_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r02l_bench_default.log 2>&1 || exit $?
for r in 1 2; do
for c in 10000 1250; do
for a in "--variant 0" "--variant 3" "--variant 3 --no-fused"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 3 --cells $c $a > gpurun_out/r02l_b.log 2>&1 || exit $?
  echo "$r $c $a $(tail -1 gpurun_out/r02l_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "LT", d["config"]["bins_per_tile"])')" >> gpurun_out/r02l_ab.log
done
done
done
