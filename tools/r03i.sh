set -o pipefail
timeout -k 10 500 python -u tools/genome_mode_probe.py > gpurun_out/r03i_mode_probe.log 2>&1 || { tail -20 gpurun_out/r03i_mode_probe.log; exit 1; }
grep '^{' gpurun_out/r03i_mode_probe.log
for round in 1 2; do
  for prior in g1_clones g1_composite; do
    timeout -k 10 200 python bench.py --prior $prior --no-cpu-baseline > gpurun_out/r03i_bench_${prior}_$round.log 2>&1 || { tail -20 gpurun_out/r03i_bench_${prior}_$round.log; exit 1; }
    echo "$round $prior $(tail -1 gpurun_out/r03i_bench_${prior}_$round.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), d["config"].get("cn_prior"))')"
  done
done
