#!/bin/bash
# Round-4 GPU session 16: p9 = per-launch staged rows for one group of 16-lane segments only --
# full GPU tests, A/B against the committed library (cur) on medium @ 4,096 and large @ 8,192.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s16.log 2>&1 || { tail -30 gpurun_out/pytest_s16.log; exit 1; }
tail -1 gpurun_out/pytest_s16.log
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="p9 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=8192 VARIANTS="p9 cur" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
