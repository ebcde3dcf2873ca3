#!/bin/bash
# Round-5 session: heterogeneous-table tests on the in-tree library (mode 6), then interleaved
# A/B of the heterogeneous table forms (m6: 4-bit station map, m5: u16 cell entries) with one
# and two groups per wavefront, against HEAD's packed kernel (base).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu -k "reward_exact or heterogeneous or mixed" \
  --timeout 150 --timeout-method thread > gpurun_out/pytest_het.log 2>&1 \
  || { echo "pytest het failed"; tail -60 gpurun_out/pytest_het.log; exit 1; }
tail -2 gpurun_out/pytest_het.log
WL=mobile-large-mixed-v0 VARIANTS="base m6 m6@two_groups=1 m5 m5@two_groups=1" REPS=2 LENS="20 200" \
  bash tools/ab.sh > /dev/null || exit 1
WL=mobile-medium-central-v0 E=4096 VARIANTS="base m6" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-custom-128x1024-v0 E=1024 VARIANTS="base m6" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-small-central-v0 E=65536 VARIANTS="base m6" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
VARIANTS="base m6" REPS=2 LENS="1 20 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
