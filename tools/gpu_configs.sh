#!/bin/bash
# Every BASELINE.json single-GPU config and the per-env-layout paths on one box (run from the repo
# root on the GPU box): rocprofv3 profiles (tools/profile.sh) of the custom 128x1024 and
# per-env-layout rollout launches, bench lines of each workload, the layout-scoring bench.
# Every GPU step has its own time limit; the first failure ends the script.
#   PROFILE_TAG (default r02): profile summaries <tag>_custom, <tag>_perenv
#   SKIP_PROFILE=1: bench lines only
set -o pipefail
mkdir -p gpurun_out
TAG=${PROFILE_TAG:-r02}
export TMPDIR=/tmp
CUSTOM="--workload mobile-custom-128x1024-v0 --envs 1024"
PERENV="--workload mobile-large-perenv-v0 --envs 65536"
if [ -z "$SKIP_PROFILE" ]; then
  tools/profile.sh ${TAG}_custom $CUSTOM || exit 1
  tools/profile.sh ${TAG}_perenv $PERENV || exit 1
  python tools/merge_profiles.py || exit 1
fi
i=0
for b in "$CUSTOM" "$PERENV" "--workload mobile-medium-central-v0 --envs 4096" \
         "--workload mobile-large-ma-v0 --envs 32768" "--workload mobile-small-central-v0 --envs 65536" \
         "--engine scenario_constants=-1"; do  # (the last: the headline on the generic instance)
  timeout -k 10 300 python bench.py $b --no-cpu-baseline > gpurun_out/bench_cfg_$i.log 2>&1 \
    || { echo "bench $b failed"; tail -30 gpurun_out/bench_cfg_$i.log; exit 1; }
  echo "== $b"; tail -1 gpurun_out/bench_cfg_$i.log
  i=$((i+1))
done
timeout -k 10 300 python tools/bench_scoring.py --layouts 100000 > gpurun_out/bench_scoring.log 2>&1 \
  || { echo "bench_scoring failed"; tail -30 gpurun_out/bench_scoring.log; exit 1; }
tail -1 gpurun_out/bench_scoring.log
