#!/bin/bash
# Parity lease (tools/r04h.sh), then A/Bs on the same box: the build before the site-value
# rounding (ab/libpert_e6e.so) and write-through streamed stores (ab/libpert_cpol19.so).
set -o pipefail
TAG=${1:-r04m}
bash tools/r04h.sh $TAG || exit 1
bash tools/ab_bench.sh ${TAG}_e6e ab/libpert_e6e.so || exit 1
bash tools/ab_bench.sh ${TAG}_cpol19 ab/libpert_cpol19.so || exit 1
