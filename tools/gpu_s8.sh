#!/bin/bash
# Round-4 GPU session 8: the software-pipelined one-group rollout (two_groups=3) -- its GPU
# tests, then medium @ 4,096 and large @ 4,096 rollouts interleaved against the packed kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 150 --timeout-method thread -k "forced_shapes or pipelined" > gpurun_out/pytest_s8.log 2>&1 || { tail -40 gpurun_out/pytest_s8.log; exit 1; }
tail -1 gpurun_out/pytest_s8.log
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="cur cur@two_groups=3 cur@two_groups=2" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=8192 VARIANTS="cur cur@two_groups=3" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
