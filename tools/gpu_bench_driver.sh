#!/bin/bash
# Dev: the driver's bench shape (--steps 20 --warmup 5) a few times, with repeated timed regions;
# REH: the --rehearsals values to interleave.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for reh in ${REH:-20}; do
    echo "rehearsals $reh" >> gpurun_out/bench_driver.log
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --timed-repeats ${REPS:-30} --rehearsals $reh ${BENCH_ARGS} \
      >> gpurun_out/bench_driver.log 2>&1 || exit 1
  done
done
python - <<'PY'
import json
reh = None
for ln in open("gpurun_out/bench_driver.log"):
    if ln.startswith("rehearsals"):
        reh = ln.split()[1]
    if ln.startswith("{"):
        d = json.loads(ln)
        r = sorted(d.get("timed_repeats_ms", []))
        print("reh", reh, round(d["ms_per_step"] * 20e3, 1), "us first;", "repeats min/med/max us:",
              [round(x * 1e3, 1) for x in (r[0], r[len(r) // 2], r[-1])] if r else None,
              "events", round(d["roofline"]["launch_ms"] * 1e3, 1))
PY
