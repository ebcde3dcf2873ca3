#!/bin/bash
# Round-4 GPU session 18: shorter staging windows of the two-group rollout (2 / 4 / 6 / 8 rows)
# vs the default 47, interleaved; then medium and the per-env layouts' kernel at 8 rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
VARIANTS="cur@stage_rows=8 cur@stage_rows=2 cur@stage_rows=4 cur@stage_rows=6 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=4096 WL=mobile-medium-central-v0 VARIANTS="cur cur@stage_rows=8" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-large-perenv-v0 VARIANTS="cur cur@stage_rows=8" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
