#!/bin/bash
# Round-5 session: the GPU suite + smoke on the in-tree library, then interleaved A/B of the final
# guard (fin) against HEAD~4 (base) and the all-integer tests (thr).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
VARIANTS="base fin thr" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-medium-central-v0 E=4096 VARIANTS="base fin thr" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-custom-128x1024-v0 E=1024 VARIANTS="base fin" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
