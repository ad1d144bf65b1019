#!/bin/bash
# This tree's libpert_hip built with extra compile definitions, for an in-lease A/B
# (PERT_LIB=<out> python bench.py ...):   bash tools/build_variant_lib.sh OUT.so -DNAME=VALUE ...
# e.g. -DPERT_SHIFT_N=4 (round 5's small-delta threshold).  Built here, shipped with the tree.
set -euo pipefail
OUT=$1; shift
R=$(pwd)
T=$(mktemp -d)
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -fno-signed-zeros -I $R/include $*"
for f in pert_kernels tau_kernels pert_comm; do
  $HIPCC -c $R/scdna_replication_tools_amd/csrc/$f.hip -o $T/$f.o &
done
wait
echo "const char* pert_version(void) { return \"pert_hip variant gfx950 src=variant $*\"; }" > $T/v.c
gcc -O2 -fPIC -c $T/v.c -o $T/v.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/*.o -o $OUT
rm -rf $T
