#!/bin/bash
# Round-4 GPU session 14: the WIP kernels of branch wip-r04-lds2 as libmev_p7.so (p7 = p6 + the
# tables' LDS-DMA overlapped with the first step's movement; p6 = per-wave areas after the
# mode-3 rates in use and a launch's staged rows flushed once at its end where they fit; p5 =
# the pipelined kernel with constant masks): the full GPU tests against p7 (MEV_LIB), then
# interleaved A/B against the committed library (cur).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cp mobile-env-gan_amd/lib/libmev.so mobile-env-gan_amd/lib/libmev_cur.so
MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_p7.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s14.log 2>&1 || { tail -30 gpurun_out/pytest_s14.log; exit 1; }
tail -1 gpurun_out/pytest_s14.log
rm -f gpurun_out/ab.log
VARIANTS="p7 p6 cur" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=4096 WL=mobile-medium-central-v0 VARIANTS="p7 p5 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
