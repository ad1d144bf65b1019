#!/bin/bash
# Build this tree's libpert_hip with extra preprocessor definitions, for A/B timing:
#   tools/build_def.sh OUT.so -DPERT_FIN_U=8 ...      then   PERT_LIB=OUT.so python bench.py ...
set -euo pipefail
OUT=$1; shift
R=$(pwd)
T=$(mktemp -d)
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -fno-signed-zeros"
$HIPCC "$@" -I $R/include -c $R/scdna_replication_tools_amd/csrc/pert_kernels.hip -o $T/k.o
$HIPCC -I $R/include -c $R/scdna_replication_tools_amd/csrc/tau_kernels.hip -o $T/tau.o
$HIPCC -I $R/include -c $R/scdna_replication_tools_amd/csrc/pert_comm.hip -o $T/comm.o
echo "const char* pert_version(void) { return \"pert_hip def gfx950 $*\"; }" > $T/v.c
gcc -O2 -fPIC -c $T/v.c -o $T/v.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/k.o $T/tau.o $T/comm.o $T/v.o -o $OUT
rm -rf $T
