#!/bin/bash
# Round-2 GPU session (run on the GPU box from the repo root): GPU tests, smoke, rocprofv3 profile
# of the bench's rollout launch and of the one-step launch, then the bench. Every GPU step has its
# own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${PROFILE_TAG:-r02}
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ -z "$SKIP_PROFILE" ]; then
  tools/profile.sh $TAG || exit 1
  tools/profile.sh ${TAG}_single --launch single || exit 1
  python tools/merge_profiles.py || exit 1  # (the box's copy: the bench reads it)
fi
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; cat gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_driver.log 2>&1 || { echo bench20 failed; cat gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log
