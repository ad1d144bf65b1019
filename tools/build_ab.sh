#!/bin/bash
# Build libpert_hip from another git revision's kernel sources (same C ABI) for A/B timing:
#   tools/build_ab.sh REV OUT.so      then   PERT_LIB=OUT.so python bench.py ...
# The revision's pert_kernels.hip (+ its pert_math.h / pert_hip.h) is linked with this tree's
# tau_kernels.hip and a pert_version() stub where the revision lacks them, so the A/B library
# exports every symbol _native.py checks.
set -euo pipefail
REV=$1; OUT=$2
R=$(pwd)
T=$(mktemp -d)
mkdir -p $T/include $T/csrc
git show $REV:include/pert_hip.h > $T/include/pert_hip.h
git show $REV:scdna_replication_tools_amd/csrc/pert_kernels.hip > $T/csrc/pert_kernels.hip
git show $REV:scdna_replication_tools_amd/csrc/pert_math.h > $T/csrc/pert_math.h
sed -i 's#"../../include/pert_hip.h"#"../include/pert_hip.h"#' $T/csrc/pert_kernels.hip
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -fno-signed-zeros"
$HIPCC -I $T/include -c $T/csrc/pert_kernels.hip -o $T/k.o
OBJS="$T/k.o"
if ! grep -q "pert_tau_kmeans_em" $T/include/pert_hip.h; then
  $HIPCC -I $R/include -c $R/scdna_replication_tools_amd/csrc/tau_kernels.hip -o $T/tau.o
  OBJS="$OBJS $T/tau.o"
fi
if ! grep -q "const char\* pert_version(void) {" $T/csrc/pert_kernels.hip; then
  echo "const char* pert_version(void) { return \"pert_hip ab gfx950 src=$REV\"; }" > $T/v.c
  gcc -O2 -fPIC -c $T/v.c -o $T/v.o
  OBJS="$OBJS $T/v.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o $OUT
rm -rf $T
