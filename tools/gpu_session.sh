#!/bin/bash
# GPU session script (dev): tests, smoke, bench, rocprof kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; cat gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tools/profile.sh ${PROFILE_TAG:-dev} || exit 1
tools/profile.sh ${PROFILE_TAG:-dev}_single --launch single || exit 1

