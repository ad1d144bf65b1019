#!/bin/bash
# Parity lease (tools/r04h.sh) and the A/B of the default build against ab/libpert_e6e.so (the
# build before the site-value rounding) on the same box.
set -o pipefail
TAG=${1:-r04k}
bash tools/r04h.sh $TAG || exit 1
bash tools/ab_bench.sh $TAG ab/libpert_e6e.so || exit 1
