#!/bin/bash
# dev: XCD block remap on/off (timing only)
set -o pipefail
for xr in 0 1 0 1; do
  MEV_XCD_REMAP=$xr TAG=xcd$xr timeout -k 10 120 python tools/variant_bench.py 2>/dev/null || { echo "xcd $xr failed"; exit 1; }
done
