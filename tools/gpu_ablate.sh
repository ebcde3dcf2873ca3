#!/bin/bash
# dev: price each phase of the step kernel with ablated builds (timing only)
set -o pipefail
for lib in ${LIBS:-libmev ablate_compute_only ablate_no_draw ablate_no_pairwise ablate_no_move ablate_no_rate ablate_no_util ablate_all libmev}; do
  MEV_VB_CASES=2 TAG=$lib MEV_LIB=$PWD/mobile-env-gan_amd/lib/$lib.so timeout -k 10 120 python tools/variant_bench.py 2>/dev/null || { echo "variant $lib failed"; exit 1; }
done
timeout -k 10 120 python tools/membench.py
