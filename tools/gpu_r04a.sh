#!/bin/bash
# Round-4 GPU session A: the GPU test suite, 20-step timeline probe, kernel-variant A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail=10 --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_r04a.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_r04a.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=5 timeout -k 10 150 python -u tools/ts_probe.py 20 > gpurun_out/ts_new.log 2>&1 || exit 1
SINGLE=1 VARIANTS="${VARIANTS:-cur wflush trim cur@compact_state=-1 sc1}" REPS=2 LENS="20 200" bash tools/ab.sh || exit 1
SINGLE=1 E=1024 WL=mobile-custom-128x1024-v0 VARIANTS="cur blk cur@compact_state=-1" REPS=2 LENS="200" bash tools/ab.sh || exit 1
E=4096 WL=mobile-medium-central-v0 VARIANTS="cur pcnt" REPS=2 LENS="20 200" bash tools/ab.sh || exit 1
WL=mobile-large-mixed-v0 VARIANTS="cur sc1" REPS=2 LENS="200" bash tools/ab.sh
