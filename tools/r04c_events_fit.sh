set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04c_events.log; : > $O
for args in "" "--cells 1250"; do
  for es in 1 8 0; do
    timeout -k 10 150 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --event-stride $es $args > gpurun_out/r04c.tmp 2>&1 || { tail -5 gpurun_out/r04c.tmp; exit 1; }
    python -c "
import json; r=json.loads(open('gpurun_out/r04c.tmp').read().strip().splitlines()[-1]); rf=r['roofline']
print('cells', r['config']['cells'], 'event_stride $es', 'step_ms', round(r['ms_per_step'],4), 'pass_ms', round(rf['kernel_ms'],4), 'ceiling', round(rf['pattern_ceiling']['ms'],4))" | tee -a $O
  done
done
timeout -k 10 300 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r04c_fullfit_c4.json 2> gpurun_out/r04c_fullfit_c4.err || { tail -5 gpurun_out/r04c_fullfit_c4.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/r04c_fullfit_c4.json').read().strip().splitlines()[-1])
t=d['timings_s']; print(t['phases']); print('ms_per_step', d['ms_per_step'], 'total', t['total'])"
