#!/bin/bash
# GPU session script (dev): tests, smoke, rocprof profile of the bench launches, then the bench
# (which reads the profile summary written on the same box: rocprof time and PMC traffic).
# Afterwards, locally: python tools/pmc_summary.py gpurun_out/prof_TAG TAG "<args>" for both
# launch shapes (the same files), and copy gpurun_out/bench.log's last line to profiles/.
set -o pipefail
mkdir -p gpurun_out
TAG=${PROFILE_TAG:-dev}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
tools/profile.sh $TAG || exit 1
tools/profile.sh ${TAG}_single --launch single || exit 1
python tools/pmc_summary.py gpurun_out/prof_$TAG $TAG "--profile-run --steps 1000 --warmup 1000" > /dev/null || exit 1
python tools/pmc_summary.py gpurun_out/prof_${TAG}_single ${TAG}_single "--profile-run --steps 1000 --warmup 1000 --launch single" > /dev/null || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; cat gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
