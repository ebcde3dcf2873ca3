#!/bin/bash
# A/B: the two-group step's risky test as one unsigned compare with the rare overwrite (v2)
# against the committed form (fin), 65,536 large envs and 4,096 medium (tools/ab.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
VARIANTS="fin v2" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-large-ma-v0 E=32768 VARIANTS="fin v2" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
