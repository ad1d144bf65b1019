#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/guess_times_profile.py --cells 10000 > gpurun_out/r02v_guess.log 2>&1 || exit $?
tail -1 gpurun_out/r02v_guess.log
timeout -k 10 900 bash tools/r02u.sh || exit $?
