#!/bin/bash
# Session 25: block kernel one-step prologue -- the culling-record flag loaded with the state
# (rok), plus the one-step draw window in LDS (rokw, = the working tree): block parity, then
# interleaved A/B vs HEAD for custom 128x1024 (1,024 envs) one-step and 200-step launches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "block or custom or het or wide" > gpurun_out/s25_tests.log 2>&1 || { tail -30 gpurun_out/s25_tests.log; exit 1; }
tail -2 gpurun_out/s25_tests.log
rm -f gpurun_out/ab.log
E=1024 WL=mobile-custom-128x1024-v0 SINGLE=1 VARIANTS="base rok rokw" REPS=4 LENS="200" bash tools/ab.sh || exit 1
echo done
