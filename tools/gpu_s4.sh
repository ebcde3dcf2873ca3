#!/bin/bash
# Round-4 GPU session 4: does the odd-XCD slowness follow the XCD or the env range it writes?
# Per-wave phase stamps with the XCD-contiguous ranges as usual, rotated by 1 and 4 XCDs, and
# without the remap.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rm in 0 2 5 -1 0; do
  MEV_ENGINE=xcd_remap=$rm MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=2 timeout -k 10 150 python -u tools/ts_probe.py 20 200 > gpurun_out/ts_tmp.log 2>&1 || { tail gpurun_out/ts_tmp.log; exit 1; }
  sed "s/^{/{\"remap\": $rm, /" gpurun_out/ts_tmp.log | grep '^{' >> gpurun_out/ts_s4.log
done
