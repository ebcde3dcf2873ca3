#!/bin/bash
# dev: parity tests, then time the packed kernel in its launch modes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
MEV_PERSISTENT=2 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu_p.log 2>&1 || { echo "pytest persistent failed"; tail -40 gpurun_out/pytest_gpu_p.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_p.log
for p in ${PERS:-0 1 2 4 8}; do
  MEV_PERSISTENT=$p TAG="persistent=$p" MEV_VB_CASES=${CASES:-2} timeout -k 10 120 python tools/variant_bench.py 2>/dev/null || { echo "variant $p failed"; exit 1; }
done
