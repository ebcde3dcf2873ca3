#!/bin/bash
# Round-4 GPU session 15: p8 = the committed kernels with k_steps_lds2's staged rows sized for the
# launch's own waves (full GPU tests), A/B against the committed library (cur) and p7.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s15.log 2>&1 || { tail -30 gpurun_out/pytest_s15.log; exit 1; }
tail -1 gpurun_out/pytest_s15.log
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="p8 cur p7" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
VARIANTS="p8 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=8192 VARIANTS="p8 cur" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
