#!/bin/bash
# Round-4 GPU session 5: XCD balance of the two-group rollout -- GPU tests, interleaved A/B
# (balanced / equal contiguous ranges / the previous commit's tile order), per-XCD wave ends.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s5.log 2>&1 || { tail -30 gpurun_out/pytest_s5.log; exit 1; }
tail -1 gpurun_out/pytest_s5.log
rm -f gpurun_out/ab.log
SINGLE= VARIANTS="cur cur@xcd_remap=9 old" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=3 timeout -k 10 150 python -u tools/ts_probe.py 20 200 > gpurun_out/ts_s5.log 2>&1 || { tail gpurun_out/ts_s5.log; exit 1; }
MEV_ENGINE=xcd_remap=9 MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=2 timeout -k 10 150 python -u tools/ts_probe.py 20 200 > gpurun_out/ts_s5_eq.log 2>&1 || { tail gpurun_out/ts_s5_eq.log; exit 1; }
