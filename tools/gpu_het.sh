#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "heterogeneous or wide_map" > gpurun_out/pytest_het.log 2>&1 \
  || { echo "pytest het failed"; tail -60 gpurun_out/pytest_het.log; exit 1; }
tail -3 gpurun_out/pytest_het.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_shipped.py -k mixed > gpurun_out/pytest_mixed.log 2>&1 \
  || { echo "pytest mixed failed"; tail -60 gpurun_out/pytest_mixed.log; exit 1; }
tail -2 gpurun_out/pytest_mixed.log
for v in "" two_groups=2 two_groups=-1 ""; do
  MEV_ENGINE=$v WL=mobile-large-mixed-v0 timeout -k 10 120 python tools/launch_len.py 20 200 \
    > gpurun_out/ll_mixed.log 2>&1 || { echo "launch_len $v failed"; cat gpurun_out/ll_mixed.log; exit 1; }
  echo "variant [$v]"; grep '^{' gpurun_out/ll_mixed.log
done
