#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "heterogeneous or mixed or velocit" --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_het.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_het.log; exit 1; }
tail -2 gpurun_out/pytest_het.log
WL=mobile-large-mixed-v0 VARIANTS="base nov15" REPS=3 LENS="1 20 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
