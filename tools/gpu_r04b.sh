#!/bin/bash
# Round-4 GPU session B: committed profiles (tools/profile.sh: kernel trace + separate PMC passes)
# of every launch shape the verdict asks about, then the bench lines (default run, the driver's
# --steps 20 --warmup 5 shape, each workload). The first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${R:-r04}
CUSTOM="--workload mobile-custom-128x1024-v0 --envs 1024"
bash tools/profile.sh ${R}_driver --chunk 20 || exit 1
bash tools/profile.sh ${R} || exit 1
bash tools/profile.sh ${R}_single --launch single || exit 1
bash tools/profile.sh ${R}_custom $CUSTOM || exit 1
bash tools/profile.sh ${R}_custom_single $CUSTOM --launch single || exit 1
bash tools/profile.sh ${R}_medium --workload mobile-medium-central-v0 --envs 4096 || exit 1
bash tools/profile.sh ${R}_mixed --workload mobile-large-mixed-v0 || exit 1
python3 tools/merge_profiles.py gpurun_out/profiles > /dev/null || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${R}_driver.json 2> gpurun_out/bench_${R}_driver.err || exit 1
tail -c 600 gpurun_out/bench_${R}_driver.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_${R}.json 2> gpurun_out/bench_${R}.err || exit 1
tail -c 300 gpurun_out/bench_${R}.json
echo done
