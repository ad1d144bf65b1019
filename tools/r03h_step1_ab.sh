set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loop.py tests/test_gpu_edge.py tests/test_gpu_chain.py -k "step1 or chain and not genome" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_tests.log 2>&1 || { tail -40 gpurun_out/r03h_tests.log; exit 1; }
tail -3 gpurun_out/r03h_tests.log
for round in 1 2; do
  for L in libpert_hip.so libpert_ab_r03c.so; do
    PERT_LIB=$(pwd)/scdna_replication_tools_amd/$L timeout -k 10 200 python bench.py --fit step1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r03h_ab_${L}_$round.log 2>&1 || exit 1
    echo "$round $L $(tail -1 gpurun_out/r03h_ab_${L}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4))')"
  done
done
PERT_DUMP_DIR=gpurun_out timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -k genome -x -v -s --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_genome.log 2>&1
tail -5 gpurun_out/r03h_genome.log
