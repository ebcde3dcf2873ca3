#!/bin/bash
# dev: parity tests, then time kernel variants (single-group vs persistent) and the memory floor
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
MEV_PACKED_MODE=persistent timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu_p.log 2>&1 || { echo "pytest persistent failed"; tail -40 gpurun_out/pytest_gpu_p.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_p.log
timeout -k 10 120 python tools/membench.py || exit 1
for mode in single persistent; do
  for bpc in ${BPCS:-0}; do
    if [ $bpc = 0 ]; then unset MEV_PERSISTENT_BLOCKS_PER_CU; else export MEV_PERSISTENT_BLOCKS_PER_CU=$bpc; fi
    MEV_PACKED_MODE=$mode TAG="$mode bpc=$bpc" timeout -k 10 120 python tools/variant_bench.py 2>/dev/null || { echo "variant $mode $bpc failed"; exit 1; }
  done
done
