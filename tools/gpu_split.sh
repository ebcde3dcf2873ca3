#!/bin/bash
# dev: single-stream vs two-half launch shape, same library (timing only)
set -o pipefail
for sp in 1 2 1 2; do
  MEV_VB_SPLIT=$sp timeout -k 10 120 python tools/variant_bench.py 2>/dev/null || { echo "split $sp failed"; exit 1; }
done
