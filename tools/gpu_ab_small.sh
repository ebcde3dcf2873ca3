#!/bin/bash
# Variants built first with tools/build_variant.sh (pre = before the guard, cur = HEAD, late =
# the packed kernels' exact-reward branch after the step's stores):
# the GPU tests on the in-tree library, then interleaved A/Bs (tools/ab.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_late.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_late.log; exit 1; }
tail -2 gpurun_out/pytest_late.log
WL=mobile-small-central-v0 VARIANTS="pre cur late" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
SINGLE=1 WL=mobile-large-central-v0 VARIANTS="cur late" REPS=3 LENS="20" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r.get("b2b_ms"))
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v if x is not None))
PY
