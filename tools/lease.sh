#!/bin/bash
# One GPU lease, parametrised (replaces the per-lease tools/r0*.sh scripts of rounds 4-5).
# Run on the GPU box from the repo root:
#   gpurun -- 'bash tools/lease.sh TAG STEP [STEP ...]'
# Every step runs under its own time limit and writes under gpurun_out/TAG/; the first step
# that fails (test failure, time limit, fault) ends the lease -- no further GPU step runs.
# Steps:
#   gpu-tests        the whole -m gpu suite (as the driver runs it)
#   tests:FILE[,..]  the named test files only (e.g. tests:test_gpu_native_comm_ranks.py)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (C4, K = 200)
#   bench-k20        the driver's settings (--steps 20 --warmup 5)
#   bench-c5         C5 (configs[4]) with --steps 20
#   trace            rocprofv3 --kernel-trace --stats of the default bench
#   pmc              tools/profile.sh's counter passes (one --pmc run each) + summary
#   shard-table      tools/shard_runs.sh + shard_table.py (per-rank shards of C4 / C5 against the whole step)
#   overlap-ab       tools/overlap_ab.sh (the sharded step's all-reduce overlap, with a 20 us stand-in)
#   fullfit-c4       tools/fullfit_bench.py --config c4
#   fullfit-c1       bench.py --fullfit-c1
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
T="timeout -k 10"
PYT="python -u -m pytest -x -v -rP --timeout 150 --timeout-method thread"
for STEP in "$@"; do
  echo "[lease $TAG] $STEP $(date +%T)"
  case $STEP in
    gpu-tests) $T 900 $PYT -m gpu tests > "$OUT/gpu_tests.log" 2>&1 ;;
    tests:*) FILES=$(echo "${STEP#tests:}" | tr ',' '\n' | sed 's|^|tests/|' | tr '\n' ' ')
             $T 900 $PYT $FILES > "$OUT/tests_$(echo "${STEP#tests:}" | tr ',/' '__').log" 2>&1 ;;
    smoke) $T 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 ;;
    bench) $T 400 python bench.py > "$OUT/bench.log" 2>&1 ;;
    bench-k20) $T 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.log" 2>&1 ;;
    bench-c5) $T 400 python bench.py --config c5 --steps 20 --no-cpu-baseline > "$OUT/bench_c5.log" 2>&1 ;;
    trace) (cd /tmp && export TMPDIR=/tmp && $T 400 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/trace.log" 2>&1) ;;
    pmc) $T 1000 bash tools/profile.sh "$TAG" ;;
    overlap-ab) $T 1100 bash tools/overlap_ab.sh "$TAG" 2 > "$OUT/overlap_ab.log" 2>&1 ;;
    shard-table) $T 900 bash tools/shard_runs.sh "$TAG" 2 > "$OUT/shard_table.log" 2>&1 ;;
    fullfit-c4) $T 400 python tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > "$OUT/fullfit_c4.json" \
                  2> "$OUT/fullfit_c4.log" ;;
    fullfit-c1) $T 300 python bench.py --fullfit-c1 > "$OUT/fullfit_c1.log" 2>&1 ;;
    *) echo "unknown step $STEP" >&2; exit 2 ;;
  esac
done
echo "[lease $TAG] done $(date +%T)"
