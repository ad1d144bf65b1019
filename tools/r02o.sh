#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 ./tools/stream_probe 10000 5451 48 10 > gpurun_out/r02o_probe.log 2>&1 || exit $?
timeout -k 10 200 ./tools/stream_probe 1250 5451 54 20 >> gpurun_out/r02o_probe.log 2>&1 || exit $?
