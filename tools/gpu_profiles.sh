#!/bin/bash
# GPU box: the round's committed profiles (tools/profile.sh, one tag per launch shape) and the
# bench lines they feed, in two parts (each fits one gpurun call):
#   bash tools/gpu_profiles.sh ROUND 1   headline 200-step, the driver's 20-step, the Gym step,
#                                        medium @ 4,096; bench.py default + driver shape lines
#   bash tools/gpu_profiles.sh ROUND 2   mixed classes, ma, custom step(); then tools/gpu_configs.sh
#                                        (custom / per-env profiles, every config's bench line)
# -> gpurun_out/profiles/ (tools/merge_profiles.py folds them into profiles/), gpurun_out/bench*.
set -o pipefail
R=${1:-r05}
export TMPDIR=/tmp
mkdir -p gpurun_out
case ${2:-1} in
1)
  STEPS="prof bench" PROF="$R:;${R}_driver:--chunk 20;${R}_single:--launch single;${R}_medium:--workload mobile-medium-central-v0 --envs 4096" \
    bash tools/gpu_round.sh || exit 1 ;;
2)
  STEPS="prof" PROF="${R}_mixed:--workload mobile-large-mixed-v0;${R}_ma:--workload mobile-large-ma-v0 --envs 32768;${R}_custom_single:--workload mobile-custom-128x1024-v0 --envs 1024 --launch single" \
    bash tools/gpu_round.sh || exit 1
  PROFILE_TAG=$R bash tools/gpu_configs.sh || exit 1 ;;
esac
