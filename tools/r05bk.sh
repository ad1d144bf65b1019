#!/bin/bash
# Round 5, lease bk: at HEAD (init quantiles, shipped trajectory) -- GPU suite, smoke, the default bench line.
set -o pipefail
TAG=${1:-r05bk}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
python -c "
import json; d=json.load(open('gpurun_out/parity_report.json')); g=d.get('genome_chain_64x64x5451',{})
print('chain stops', {k: v['product'] for k, v in g.get('stops', {}).items()})"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_bench.log | python -c "
import json,sys; r=json.loads(sys.stdin.read()); rf=r['roofline']
print('C4 value %.4g ms/step %.4f evented %.4f kernel %.4f ceil %.4f frac %.3f cpu %.4g place %s' % (r['value'], r['ms_per_step'], r['ms_per_step_evented'], rf['kernel_ms'], rf['pattern_ceiling']['ms'], rf['frac'], r['cpu_baseline']['value'], rf.get('pi_placement',{}).get('candidates_ms')))"
exit $rc
