#!/bin/bash
# Round-4 GPU session 17: staging-window length of the two-group rollout (stage_rows cap:
# flushes -- and workgroup barriers -- every 8 / 16 / 24 rows vs the default 47), interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
VARIANTS="cur cur@stage_rows=8 cur@stage_rows=16 cur@stage_rows=24" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
