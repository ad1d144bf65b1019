#!/bin/bash
# Build libpert_hip from another git revision's kernel sources (same C ABI) for A/B timing:
#   tools/build_ab.sh REV OUT.so      then   PERT_LIB=OUT.so python bench.py ...
set -euo pipefail
REV=$1; OUT=$2
T=$(mktemp -d)
mkdir -p $T/include $T/csrc
git show $REV:include/pert_hip.h > $T/include/pert_hip.h
git show $REV:scdna_replication_tools_amd/csrc/pert_kernels.hip > $T/csrc/pert_kernels.hip
git show $REV:scdna_replication_tools_amd/csrc/pert_math.h > $T/csrc/pert_math.h
sed -i 's#"../../include/pert_hip.h"#"../include/pert_hip.h"#' $T/csrc/pert_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I $T/include $T/csrc/pert_kernels.hip -o $OUT
rm -rf $T
