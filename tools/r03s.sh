set -o pipefail
for round in 1 2; do
  for lt in 0 32 48 64 80; do
    timeout -k 10 200 python bench.py --fit step1 --steps 50 --warmup 5 --no-cpu-baseline --bins-per-tile $lt > gpurun_out/r03s.log 2>&1 || { tail -20 gpurun_out/r03s.log; exit 1; }
    echo "$round lt=$lt $(tail -1 gpurun_out/r03s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(d["roofline"]["kernel_ms"],4), "lt", d["config"]["bins_per_tile"])')"
  done
done
