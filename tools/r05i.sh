#!/bin/bash
# Round 5, lease i: smoke, then the roofline evidence of the headline pass at HEAD from one lease
# (kernel trace + PMC passes + the bench --profile line; pmc_traffic.json regenerated).
set -o pipefail
TAG=${1:-r05i}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash tools/roofline_evidence.sh $TAG
