#!/bin/bash
# Round-4 GPU session 7: timing ablation -- env-major trajectory rows vs step-major (results not
# checked), interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab.log
VARIANTS="em base" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
