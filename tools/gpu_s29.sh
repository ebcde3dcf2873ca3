#!/bin/bash
# Session 29: round-4 profiles of the remaining bench workloads (tools/profile.sh: kernel trace +
# separate PMC passes): custom 128x1024 (re-run: the summary now names the launch's own kernel
# instance), per-env layouts, large-ma, small.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/profiles
bash tools/profile.sh r04_custom --workload mobile-custom-128x1024-v0 --envs 1024 || exit 1
bash tools/profile.sh r04_perenv --workload mobile-large-perenv-v0 --envs 65536 || exit 1
bash tools/profile.sh r04_ma --workload mobile-large-ma-v0 --envs 32768 || exit 1
bash tools/profile.sh r04_small --workload mobile-small-central-v0 --envs 65536 || exit 1
echo done
