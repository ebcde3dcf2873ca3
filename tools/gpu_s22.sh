#!/bin/bash
# Session 22: the whole GPU suite and smoke() on main (the round-end driver's checks).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests \
  > gpurun_out/s22_tests.log 2>&1 || { tail -40 gpurun_out/s22_tests.log; exit 1; }
tail -3 gpurun_out/s22_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s22_smoke.log 2>&1 || { tail -20 gpurun_out/s22_smoke.log; exit 1; }
tail -3 gpurun_out/s22_smoke.log
