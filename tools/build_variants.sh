#!/bin/bash
# P=13-only builds of the current kernel sources with compile-time knobs, for A/B timing:
#   tools/build_variants.sh NAME "-DKNOB=V ..." [NAME "-D..."] ...   -> scdna_replication_tools_amd/ab_NAME.so
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  NAME=$1; DEFS=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -fno-slp-vectorize -fno-signed-zeros -DPERT_ONLY_P13 \
    -DPERT_SOURCE_HASH="\"ab-$NAME\"" $DEFS -I "$R/include" "$R/scdna_replication_tools_amd/csrc/pert_kernels.hip" \
    -o "$R/scdna_replication_tools_amd/ab_$NAME.so" &
done
wait
