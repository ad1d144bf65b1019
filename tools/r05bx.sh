#!/bin/bash
# finalize_kernel duration (rocprofv3 kernel trace) with 4 / 8 / 16 partial rows in flight per thread
set -o pipefail
mkdir -p gpurun_out/r05bx
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
for L in - ab/fin8.so ab/fin16.so; do
  for c in "--cells 1250 --comm rccl" "--cells 10000"; do
    n=$(echo "$L $c" | tr -c 'a-zA-Z0-9' '_')
    if [ "$L" = - ]; then unset PERT_LIB; else export PERT_LIB=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05bx/$rep$n -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 100 $c > $GRAFT_REPO_ROOT/gpurun_out/r05bx/$rep$n.log 2>&1 || exit 1
    python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/r05bx/$rep$n/run_kernel_stats.csv')):
    if 'finalize' in r['Name'] or 'enum3' in r['Name']: print('$rep $L $c', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
" | tee -a $GRAFT_REPO_ROOT/gpurun_out/r05bx/summary.log
  done
done
done
