#!/bin/bash
# Round-4 final GPU session: the committed profiles of the final kernels (tools/profile.sh:
# kernel trace + separate PMC passes) -- the driver's 20-step launch, the 200-step bench launch,
# medium @ 4,096 -- then the bench lines (the driver's --steps 20 --warmup 5 shape, the default
# run) and every workload's line (tools/gpu_configs.sh without profiles).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r04}
bash tools/profile.sh ${R}_driver --chunk 20 || exit 1
bash tools/profile.sh ${R} || exit 1
bash tools/profile.sh ${R}_medium --workload mobile-medium-central-v0 --envs 4096 || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${R}_driver.json 2> gpurun_out/bench_${R}_driver.err || exit 1
tail -c 400 gpurun_out/bench_${R}_driver.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${R}.json 2> gpurun_out/bench_${R}.err || exit 1
tail -c 300 gpurun_out/bench_${R}.json
SKIP_PROFILE=1 bash tools/gpu_configs.sh || exit 1
echo done
