#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python tools/host_prep_cprofile.py > gpurun_out/r02x_hostprep.log 2>&1 || exit $?
head -3 gpurun_out/r02x_hostprep.log
