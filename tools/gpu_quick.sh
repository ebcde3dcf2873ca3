#!/bin/bash
# Dev GPU session: GPU tests (optionally a -k filter in $K), then bench lines given as arguments
# ("ARGS|ARGS|..."), each under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu ${K:+-k "$K"} --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
IFS='|' read -ra BENCHES <<< "$1"
i=0
for b in "${BENCHES[@]}"; do
  timeout -k 10 300 python bench.py $b > gpurun_out/bench_$i.log 2>&1 || { echo "bench $b failed"; tail -30 gpurun_out/bench_$i.log; exit 1; }
  echo "== $b"; tail -1 gpurun_out/bench_$i.log
  i=$((i+1))
done
