#!/bin/bash
# GPU box: the round's committed profiles (tools/profile.sh, one tag per launch shape) and the
# bench lines they feed (default run and the driver's `--steps 20 --warmup 5` shape).
# usage: bash tools/gpu_profiles.sh ROUND   (e.g. r03) -> gpurun_out/profiles/, gpurun_out/bench_*.json
set -o pipefail
R=${1:-r03}
mkdir -p gpurun_out
bash tools/profile.sh ${R} &&
bash tools/profile.sh ${R}_driver --chunk 20 &&
bash tools/profile.sh ${R}_single --launch single &&
python3 tools/merge_profiles.py gpurun_out/profiles > /dev/null &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${R}.json 2> gpurun_out/bench_${R}.err &&
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${R}_driver.json 2> gpurun_out/bench_${R}_driver.err &&
echo done
