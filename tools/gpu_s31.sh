#!/bin/bash
# Session 31: trajectory-store cache policy (MEV_TRAJ_AUX: default / nt / sc1) re-measured with
# the 3-row staging window, interleaved, 20 / 200-step launches at 65,536 large envs.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
VARIANTS="base nt sc1" REPS=3 LENS="20 200" bash tools/ab.sh || exit 1
echo done
