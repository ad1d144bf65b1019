#!/bin/bash
# Round 5, lease ak (placement search): the roofline evidence of the headline pass at HEAD from one lease
# (kernel trace + PMC passes + the bench --profile line; pmc_traffic.json regenerated).
set -o pipefail
TAG=${1:-r05ak}
mkdir -p gpurun_out
bash tools/roofline_evidence.sh $TAG
