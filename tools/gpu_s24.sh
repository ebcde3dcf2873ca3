#!/bin/bash
# Session 24: block kernel without scratch spills (epilogue addresses recomputed): block-kernel
# parity, then interleaved A/B vs HEAD for custom 128x1024 (1,024 envs) one-step and 200-step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "block or custom or het or wide" > gpurun_out/s24_tests.log 2>&1 || { tail -30 gpurun_out/s24_tests.log; exit 1; }
tail -2 gpurun_out/s24_tests.log
rm -f gpurun_out/ab.log
E=1024 WL=mobile-custom-128x1024-v0 SINGLE=1 VARIANTS="base nsp" REPS=4 bash tools/ab.sh || exit 1
E=1024 WL=mobile-custom-128x1024-v0 VARIANTS="base nsp" REPS=3 LENS="200" bash tools/ab.sh || exit 1
echo done
