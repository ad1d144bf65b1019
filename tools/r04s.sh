#!/bin/bash
# Kernel trace of the C1 full fit (where does a 400-cell x 271-bin step go?)
set -o pipefail
TAG=${1:-r04s}
R=$(pwd)
mkdir -p gpurun_out/prof_${TAG}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}/trace -o run --output-format csv -- python3 $R/tools/fullfit_bench.py --config c1 --cpu-sample-cells 0 > $R/gpurun_out/prof_${TAG}/fit.log 2>&1) || { tail -5 gpurun_out/prof_${TAG}/fit.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/prof_r04s/trace/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
st = collections.defaultdict(list)
for r in rows:
    st[r['Kernel_Name'][:45]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1]))[:10]:
    v.sort(); print('%-45s n %6d median %8.2f us total %8.1f ms' % (k, len(v), v[len(v)//2], sum(v)/1000))
# the steady-state period between consecutive enum3 launches
e = [int(r['Start_Timestamp']) for r in rows if 'enum3' in r['Kernel_Name']]
import statistics
d = [(b - a) / 1000 for a, b in zip(e, e[1:])]
if d: print('enum3 start-to-start median %.1f us' % statistics.median(d))
g = []
for a, b in zip(rows, rows[1:]):
    g.append((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1000)
g.sort(); print('gap median %.2f us p90 %.2f us' % (g[len(g)//2], g[int(len(g)*0.9)]))
PY
