set -o pipefail
timeout -k 10 200 python -u tools/rccl_smoke.py > gpurun_out/r03o_rccl_smoke.log 2>&1 || { tail -30 gpurun_out/r03o_rccl_smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03o_rccl_smoke.log
PERT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03o_gloo2.log 2>&1 || { tail -30 gpurun_out/r03o_gloo2.log; exit 1; }
grep '^{' gpurun_out/r03o_gloo2.log | cut -c1-400
