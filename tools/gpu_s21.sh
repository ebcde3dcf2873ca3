#!/bin/bash
# Session 21: the pipelined kernel's next cell entry read before the current step's outputs
# (parity of the pipelined launches, then interleaved A/B vs HEAD at 4,096 medium / 8,192 large).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "pipelined or two_group_kernel_forced" > gpurun_out/s21_tests.log 2>&1 || { tail -30 gpurun_out/s21_tests.log; exit 1; }
tail -2 gpurun_out/s21_tests.log
rm -f gpurun_out/ab.log
E=4096 WL=mobile-medium-central-v0 VARIANTS="base ca" REPS=4 LENS="200" bash tools/ab.sh || exit 1
E=8192 WL=mobile-large-central-v0 VARIANTS="base ca" REPS=2 LENS="200" bash tools/ab.sh || exit 1
echo done
