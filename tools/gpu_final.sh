#!/bin/bash
# Round-end rehearsal on the in-tree library: the GPU tests, smoke() and the default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_final.log; exit 1; }
tail -2 gpurun_out/pytest_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log | tail -1 | cut -c1-400
