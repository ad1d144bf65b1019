#!/bin/bash
# Round-4 parity lease (repo root on the GPU box); each step under its own limit, the first
# failure ends the script:
#   1. the genome-length chain against the fp32 oracle (product dump kept), the -m gpu suite,
#      the default bench;
#   2. pass timing with events on every / every 8th / no timed step (C4, 1,250 cells) and the
#      C4 full fit end to end.
set -o pipefail
mkdir -p gpurun_out
bash tools/r04d_parity.sh || exit 1
bash tools/r04c_events_fit.sh || exit 1
