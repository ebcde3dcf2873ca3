#!/bin/bash
# Round-4 GPU session 19: the two-group rollout's staging window at 1 / 2 / 3 / 4 rows,
# interleaved, three reps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
VARIANTS="cur@stage_rows=4 cur@stage_rows=1 cur@stage_rows=2 cur@stage_rows=3" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
