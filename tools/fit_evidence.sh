#!/bin/bash
# Evidence for the fits around the headline pass (run on the GPU box from the repo root):
#   1. bench.py --fit step1 (the observed pass, configs[3]'s 20k doubled G1/2 cells) and its
#      rocprofv3 kernel trace + PMC passes (tools/profile.sh);
#   2. the configs[0] stand-in's full fit on the GPU and on the CPU oracle (bench.py --fullfit-c1);
#   3. the C4 full fit end to end (tools/fullfit_bench.py, host prep included).
# usage: tools/fit_evidence.sh TAG [--no-profile]
set -o pipefail
TAG=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --fit step1 --steps 50 --warmup 5 --no-cpu-baseline \
  > gpurun_out/${TAG}_step1.log 2>&1 || { tail -20 gpurun_out/${TAG}_step1.log; exit 1; }
tail -1 gpurun_out/${TAG}_step1.log
if [ "$1" != "--no-profile" ]; then
  bash tools/profile.sh ${TAG}_s1 --fit step1 --steps 20 --warmup 3 --no-cpu-baseline || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/prof_${TAG}_s1/summary.json'))
for k,v in d['kernels'].items(): print(k, {x: v.get(x) for x in ('avg_ns','median_ns','warm_mean_ns','calls','hbm_bytes_per_launch')})"
fi
timeout -k 10 300 python -u bench.py --fullfit-c1 > gpurun_out/${TAG}_fullfit_c1.json 2> gpurun_out/${TAG}_fullfit_c1.err \
  || { tail -20 gpurun_out/${TAG}_fullfit_c1.err; exit 1; }
tail -c 700 gpurun_out/${TAG}_fullfit_c1.json
timeout -k 10 600 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 \
  > gpurun_out/${TAG}_fullfit_c4.json 2> gpurun_out/${TAG}_fullfit_c4.err || { tail -20 gpurun_out/${TAG}_fullfit_c4.err; exit 1; }
tail -c 900 gpurun_out/${TAG}_fullfit_c4.json
