#!/bin/bash
# A/B of the two-group step's reward guard: base (HEAD~3), new (out-of-line rare path), gi
# (inlined), ng (no in-step guard), 20- and 200-step launches at 65,536 large envs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
VARIANTS="base new gi ng" REPS=3 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
