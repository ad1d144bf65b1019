set -o pipefail
true

for round in 1 2; do
  for L in libpert_hip.so ab_head.so; do
    for cfg in "--config c5 --cells 2000 --steps 6 --warmup 2" "--steps 20 --warmup 3"; do
      PERT_LIB=$(pwd)/scdna_replication_tools_amd/$L timeout -k 10 300 python bench.py $cfg --no-cpu-baseline > gpurun_out/r03q_ab.log 2>&1 || { tail -20 gpurun_out/r03q_ab.log; exit 1; }
      echo "$round $L [$cfg] $(tail -1 gpurun_out/r03q_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_frac", round(r["pattern_ceiling"]["kernel_frac_of_ceiling"],3))')"
    done
  done
done
