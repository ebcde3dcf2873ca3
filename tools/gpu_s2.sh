#!/bin/bash
# Round-4 GPU session 2: interleaved A/B of the round-4 kernel changes at the bench's shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SINGLE=1 VARIANTS="cur c75 wgf cur@compact_state=-1" REPS=2 LENS="20 200" bash tools/ab.sh || exit 1
E=4096 WL=mobile-medium-central-v0 VARIANTS="cur c75" REPS=2 LENS="20 200" bash tools/ab.sh || exit 1
SINGLE=1 E=1024 WL=mobile-custom-128x1024-v0 VARIANTS="cur c75" REPS=2 LENS="200" bash tools/ab.sh
