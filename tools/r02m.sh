#!/bin/bash
# pattern-ceiling probe at C4 and at the 1,250-cell shard, then the default bench's rocprof evidence
mkdir -p gpurun_out
timeout -k 10 120 ./tools/stream_probe 10000 5451 48 20 > gpurun_out/r02m_probe.log 2>&1 || exit $?
timeout -k 10 120 ./tools/stream_probe 1250 5451 43 40 >> gpurun_out/r02m_probe.log 2>&1 || exit $?
timeout -k 10 1000 bash tools/profile.sh r02m || exit $?
