#!/bin/bash
# Round-4 GPU session 20: the 3-row window as the two-group default (w3) -- full GPU tests, A/B
# against the previous library (cur), then the driver's bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s20.log 2>&1 || { tail -30 gpurun_out/pytest_s20.log; exit 1; }
tail -1 gpurun_out/pytest_s20.log
rm -f gpurun_out/ab.log
VARIANTS="w3 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-large-ma-v0 E=32768 VARIANTS="w3 cur" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_s20_driver.json 2> gpurun_out/bench_s20_driver.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_s20_driver.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('launch_ms'))"
