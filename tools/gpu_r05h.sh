#!/bin/bash
# A/B: the reward guard with host-computed thresholds (thr) against the LDS-read test (new), no
# in-step guard (ng) and HEAD~4 (base), every kernel family (tools/ab.sh, interleaved).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
VARIANTS="base new thr" REPS=2 LENS="20 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-medium-central-v0 E=4096 VARIANTS="base new thr" REPS=2 LENS="200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-custom-128x1024-v0 E=1024 VARIANTS="base new thr" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
WL=mobile-small-central-v0 E=65536 VARIANTS="base new thr" REPS=2 LENS="1 200" bash tools/ab.sh > /dev/null || exit 1
python3 - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open("gpurun_out/ab.log"):
    r = json.loads(l); agg[(r["wl"], r["variant"], r["n"])].append(r["b2b_ms"])
for k, v in sorted(agg.items()): print(k, " ".join("%.4f" % x for x in v))
PY
