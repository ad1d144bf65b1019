set -o pipefail
bash tools/gpu_check.sh r03n --quick || exit 1
timeout -k 10 300 python -u bench.py --fullfit-c1 > gpurun_out/r03n_fullfit_c1.json 2> gpurun_out/r03n_fullfit_c1.err || { tail -20 gpurun_out/r03n_fullfit_c1.err; exit 1; }
timeout -k 10 400 python -u tools/fullfit_bench.py --config c4 --cpu-sample-cells 0 > gpurun_out/r03n_fullfit_c4.json 2> gpurun_out/r03n_fullfit_c4.err || { tail -20 gpurun_out/r03n_fullfit_c4.err; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/r03n_fullfit_c1.json','gpurun_out/r03n_fullfit_c4.json'):
    d=json.load(open(f)); t=d.get('timings_s', d.get('gpu_timings_s')); print(f, round(t['total'],3), t.get('phases'))"
