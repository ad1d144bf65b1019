#!/bin/bash
# Round 5, lease bw: at HEAD (placement search with the top-rate stop) -- GPU suite, smoke, the
# default bench line (tools/r05bk.sh), then the bench's N = 2 path rehearsed on one GPU (gloo).
set -o pipefail
TAG=${1:-r05bw}
bash tools/r05bk.sh $TAG || exit $?
PERT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${TAG}_gloo2.log 2>&1 || { tail -30 gpurun_out/${TAG}_gloo2.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_gloo2.log | python3 -c "
import json,sys; r=json.loads(sys.stdin.read()); print({k: r[k] for k in ('value','n_gpus','ms_per_step','scaling')}, r['config'].get('parallelism'), r['config'].get('allreduce'), r['roofline'].get('pi_placement',{}).get('candidates_ms'))"
