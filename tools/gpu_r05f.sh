#!/bin/bash
# Round-5 session: the GPU suite (the reward guard's out-of-line paths, the heterogeneous tables,
# the multi-rank tests), then interleaved A/B of the working tree (new) against HEAD~2 (base).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "reward_exact or dist or heterogeneous" \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_first.log 2>&1 \
  || { echo "pytest first failed"; tail -60 gpurun_out/pytest_first.log; exit 1; }
tail -2 gpurun_out/pytest_first.log
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
VARIANTS="base new" REPS=2 LENS="1 20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-medium-central-v0 E=4096 VARIANTS="base new" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-custom-128x1024-v0 E=1024 VARIANTS="base new" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-small-central-v0 E=65536 VARIANTS="base new" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
