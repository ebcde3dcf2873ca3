#!/bin/bash
# Session 23: timing-only A/B of one-byte serving stores (libmev_s8: -DMEV_SRV8, values not
# decoded) vs HEAD in the bench's shapes (20 / 200-step launches at 65,536 large envs).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
VARIANTS="base s8" REPS=4 LENS="20 200" bash tools/ab.sh || exit 1
echo done
