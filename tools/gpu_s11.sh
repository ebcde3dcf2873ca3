#!/bin/bash
# Round-4 GPU session 11: pipelined rollout with the split only for 16-lane segments (p3) --
# full GPU tests, A/B vs p1 (large @ 8,192 and medium @ 4,096), medium bench line + profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s11.log 2>&1 || { tail -30 gpurun_out/pytest_s11.log; exit 1; }
tail -1 gpurun_out/pytest_s11.log
rm -f gpurun_out/ab.log
E=8192 VARIANTS="p3 p1" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
E=4096 WL=mobile-medium-central-v0 VARIANTS="p3 p1" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
timeout -k 10 300 python3 bench.py --workload mobile-medium-central-v0 --envs 4096 > gpurun_out/bench_medium.json 2> gpurun_out/bench_medium.err || { tail gpurun_out/bench_medium.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_medium.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('launch_ms'))"
bash tools/profile.sh r04_medium --workload mobile-medium-central-v0 --envs 4096 || exit 1
