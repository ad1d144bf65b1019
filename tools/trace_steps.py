"""Per-step kernel timeline from a rocprofv3 kernel trace: durations of the step's kernels
and the host gap before each enumerated / observed pass.  usage: trace_steps.py run_kernel_trace.csv"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
first = [i for i, k in enumerate(ks) if "enum_dma_kernel" in k[2] or "enum_kernel" in k[2] or "obs_kernel" in k[2]]
first = first[-20:]
names = {}
gaps = []
for i in first:
    gaps.append((ks[i][0] - ks[i - 1][1]) / 1e3)
    j = i
    while j < len(ks) and (j == i or not any(t in ks[j][2] for t in ("enum_", "obs_kernel"))):
        nm = ks[j][2].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        names.setdefault(nm, []).append((ks[j][1] - ks[j][0]) / 1e3)
        j += 1
for nm, d in names.items():
    print("{:50s} mean {:8.1f} us".format(nm[:50], np.mean(d)))
print("host gap before the pass: mean {:.1f} us".format(np.mean(gaps)))
print("step period: {:.1f} us".format(np.mean(np.diff([ks[i][0] for i in first])) / 1e3))
