#!/bin/bash
# Roofline evidence of the headline pass from ONE lease (run on the GPU box from the repo root):
#   1. tools/profile.sh TAG: rocprofv3 kernel trace + separate PMC passes of bench.py (C4 step 2);
#   2. profiles/pmc_traffic.json regenerated from that PMC summary (bench.py's roofline.traffic);
#   3. bench.py --profile: the bench line with frac_trace / traffic / traffic_per_algorithmic /
#      wait_inst_frac taken from the trace and counters of step 1, same build, same box.
# usage: tools/roofline_evidence.sh TAG
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/profile.sh $TAG || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_$TAG > gpurun_out/prof_$TAG/summary.json || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_$TAG/summary.json c4 10000 gpurun_out/prof_$TAG/pmc_traffic.json || exit 1
timeout -k 10 300 python bench.py --profile gpurun_out/prof_$TAG --pmc gpurun_out/prof_$TAG/pmc_traffic.json \
  > gpurun_out/${TAG}_bench_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_profile.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_profile.log | cut -c1-1500
python3 -c "
import json
d = json.load(open('gpurun_out/prof_$TAG/summary.json'))
for k, v in d['kernels'].items():
    print(k, {x: v.get(x) for x in ('avg_ns', 'median_ns', 'warm_mean_ns', 'calls', 'hbm_bytes_per_launch')})"
