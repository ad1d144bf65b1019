#!/bin/bash
# One lease of round-4 evidence (repo root on the GPU box); each step under its own limit, the
# first failure ends the script:
#   1. the genome-length chain against the fp32 oracle (product dump kept), then the -m gpu suite;
#   2. the default bench; pass timing with events on every / every 8th / no timed step (C4, 1,250);
#   3. the C4 full fit end to end;
#   4. roofline evidence: rocprofv3 trace + PMC passes of the bench and bench.py --profile.
set -o pipefail
TAG=${1:-r04e}
mkdir -p gpurun_out
bash tools/r04d_parity.sh || exit 1
bash tools/r04c_events_fit.sh || exit 1
bash tools/roofline_evidence.sh $TAG || exit 1
