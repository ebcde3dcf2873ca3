#!/bin/bash
# Session 28: max-memory-clause scheduler vs max-ilp on the other launch shapes (one-step large,
# custom one-step / 200-step, per-env layouts), then the whole GPU suite on that build.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
V="base max_memory_clause"
SINGLE=1 VARIANTS="$V" REPS=3 LENS="20" bash tools/ab.sh || exit 1
E=1024 WL=mobile-custom-128x1024-v0 SINGLE=1 VARIANTS="$V" REPS=3 LENS="200" bash tools/ab.sh || exit 1
WL=mobile-large-perenv-v0 VARIANTS="$V" REPS=3 LENS="20 200" bash tools/ab.sh || exit 1
MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_max_memory_clause.so timeout -k 10 900 python -u -m pytest -x -q -m gpu \
  --timeout 120 --timeout-method thread tests > gpurun_out/s28_tests.log 2>&1 || { tail -30 gpurun_out/s28_tests.log; exit 1; }
tail -2 gpurun_out/s28_tests.log
echo done
