#!/bin/bash
# kernel trace of the 8-GPU shard step (1,250 cells, the library's all-reduce at world 1) with the
# placement search: where the step's time goes on a fast placement
set -o pipefail
TAG=${1:-r05aw}
R=$(pwd)
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/t -o run --output-format csv -- \
  python3 $R/bench.py --cells 1250 --comm rccl --steps 40 --warmup 5 --no-cpu-baseline > $R/gpurun_out/$TAG/bench.log 2>&1 || exit 1
cd $R
python3 - <<'PY'
import csv, glob, statistics
f = glob.glob('gpurun_out/r05aw/t/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'enum3' in r['Kernel_Name']]
st = [int(rows[i]['Start_Timestamp']) for i in idx]
print('enum3 launches', len(idx), 'median step period us', statistics.median([b - a for a, b in zip(st[50:], st[51:])]) / 1e3)
i0 = idx[60]
for r in rows[i0 - 1:i0 + 6]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print('%-50s start %8.1f dur %7.1f' % (r['Kernel_Name'][:50], (s - int(rows[i0]['Start_Timestamp'])) / 1e3, (e - s) / 1e3))
PY
