#!/bin/bash
# Round-5 committed profiles, part $1 (1: the headline shapes + bench lines; 2: the other
# workloads + the BASELINE configs' bench lines). tools/profile.sh per tag, merged by
# tools/merge_profiles.py on this side.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
case $1 in
1)
  STEPS="prof bench" PROF="r05:;r05_driver:--chunk 20;r05_single:--launch single;r05_medium:--workload mobile-medium-central-v0 --envs 4096" \
    bash tools/gpu_round.sh || exit 1 ;;
2)
  STEPS="prof" PROF="r05_mixed:--workload mobile-large-mixed-v0;r05_ma:--workload mobile-large-ma-v0 --envs 32768;r05_custom_single:--workload mobile-custom-128x1024-v0 --envs 1024 --launch single" \
    bash tools/gpu_round.sh || exit 1
  PROFILE_TAG=r05 bash tools/gpu_configs.sh || exit 1 ;;
esac
