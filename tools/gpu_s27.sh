#!/bin/bash
# Session 27: timing-only A/B of the scheduler strategy (max-ilp, the Makefile's, vs
# max-memory-clause) at 4,096 medium envs (200-step) and 65,536 large envs (20 / 200-step).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="base max_memory_clause" REPS=3 LENS="200" bash tools/ab.sh || exit 1
VARIANTS="base max_memory_clause" REPS=3 LENS="20 200" bash tools/ab.sh || exit 1
echo done
