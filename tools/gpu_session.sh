#!/bin/bash
# One GPU session on the box (run from the repo root): GPU tests (unless SKIP_TESTS), smoke,
# then the launch-length probe (tools/launch_len.py) and optional extra commands in $EXTRA.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ -z "$SKIP_LL" ]; then
  timeout -k 10 200 python tools/launch_len.py ${LL_LENS:-20 40 200} > gpurun_out/ll.log 2>&1 \
    || { echo launch_len failed; cat gpurun_out/ll.log; exit 1; }
  grep '^{' gpurun_out/ll.log
fi
if [ -n "$EXTRA" ]; then
  bash -c "$EXTRA" || { echo "extra failed"; exit 1; }
fi
