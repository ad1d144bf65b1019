#!/bin/bash
# A/B of libpert_hip builds over bench.py configurations on one box, interleaved, 2 rounds:
#   tools/ab_configs.sh "libpert_hip.so ab_other.so" "--config c5 --cells 2000 --steps 6 --warmup 2" "--steps 20 --warmup 3"
# (A/B builds: tools/build_ab.sh REV scdna_replication_tools_amd/ab_<name>.so -- names not matching
# .gpurunignore's libpert_ab_* so they travel to the box.)  Prints step / kernel ms and the
# kernel's fraction of its pattern ceiling (steps 2/3) per (round, library, configuration).
set -o pipefail
LIBS=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for L in $LIBS; do
    for cfg in "$@"; do
      PERT_LIB=$(pwd)/scdna_replication_tools_amd/$L timeout -k 10 300 python bench.py $cfg --no-cpu-baseline > gpurun_out/ab_configs.log 2>&1 || { tail -20 gpurun_out/ab_configs.log; exit 1; }
      echo "$round $L [$cfg] $(tail -1 gpurun_out/ab_configs.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; pc=r.get("pattern_ceiling") or {}; print("step_ms", round(d["ms_per_step"],4), "kernel_ms", round(r["kernel_ms"],4), "ceiling_frac", pc.get("kernel_frac_of_ceiling"), "lt", d["config"].get("bins_per_tile"))')"
    done
  done
done
