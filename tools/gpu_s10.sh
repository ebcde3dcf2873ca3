#!/bin/bash
# Round-4 GPU session 10: pipelined rollout with the draw word read a step ahead and the output
# reads split around the movement (p2) vs the committed pipelined kernel (p1) -- tests, A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 150 --timeout-method thread -k "forced_shapes or pipelined" > gpurun_out/pytest_s10.log 2>&1 || { tail -40 gpurun_out/pytest_s10.log; exit 1; }
tail -1 gpurun_out/pytest_s10.log
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="p2 p1" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=8192 VARIANTS="p2 p1" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
