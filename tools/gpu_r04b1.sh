#!/bin/bash
# Round-4 profiles, part 1 (tools/profile.sh: kernel trace + separate PMC passes): the driver's
# 20-step launch, the 200-step bench launch, the Gym step() launch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r04}
bash tools/profile.sh ${R}_driver --chunk 20 || exit 1
bash tools/profile.sh ${R} || exit 1
bash tools/profile.sh ${R}_single --launch single || exit 1
echo done
