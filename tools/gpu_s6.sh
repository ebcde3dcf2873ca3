#!/bin/bash
# Round-4 GPU session 6: the one-step kernel's draw cache -- GPU tests, then one-step launches
# interleaved against the previous commit (large 65,536 and medium 4,096 envs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s6.log 2>&1 || { tail -30 gpurun_out/pytest_s6.log; exit 1; }
tail -1 gpurun_out/pytest_s6.log
rm -f gpurun_out/ab.log
SINGLE=1 VARIANTS="nx base" REPS=3 LENS="20" bash tools/ab.sh > /dev/null || exit 1
SINGLE=1 E=4096 WL=mobile-medium-central-v0 VARIANTS="nx base" REPS=2 LENS="20" bash tools/ab.sh > /dev/null || exit 1
