#!/bin/bash
# Round-5 session: the GPU test suite, then interleaved A/B of the reward guard (new) against
# HEAD (base) on the headline, medium, custom and mixed shapes (tools/ab.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu -k "custom or block" --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_block.log 2>&1 || { echo "pytest block failed"; tail -60 gpurun_out/pytest_block.log; exit 1; }
tail -2 gpurun_out/pytest_block.log
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
VARIANTS="base new" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-medium-central-v0 E=4096 VARIANTS="base new" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-custom-128x1024-v0 E=1024 VARIANTS="base new" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-large-mixed-v0 VARIANTS="base new new@two_groups=2" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
cat gpurun_out/ab.log | cut -c1-260
