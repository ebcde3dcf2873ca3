#!/bin/bash
# Round-4 profiles, part 2: custom 128 x 1024 (rollout and step()), medium @ 4,096, mixed; then
# the bench lines (the driver's --steps 20 --warmup 5 shape and the default run).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r04}
CUSTOM="--workload mobile-custom-128x1024-v0 --envs 1024"
bash tools/profile.sh ${R}_custom $CUSTOM || exit 1
bash tools/profile.sh ${R}_custom_single $CUSTOM --launch single || exit 1
bash tools/profile.sh ${R}_medium --workload mobile-medium-central-v0 --envs 4096 || exit 1
bash tools/profile.sh ${R}_mixed --workload mobile-large-mixed-v0 || exit 1
echo done
