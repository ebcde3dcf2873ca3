#!/bin/bash
# A/B of heterogeneous-kernel variants on mobile-large-mixed-v0 (tools/ab.sh, interleaved).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
WL=mobile-large-mixed-v0 VARIANTS="${VARIANTS:-base cur}" REPS=${REPS:-3} LENS="${LENS:-20 200}" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
