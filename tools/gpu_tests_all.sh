#!/bin/bash
# The whole GPU suite without -x (every failure listed), then smoke(); each step time-limited.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread -rf ${PYTEST_ARGS} \
  > gpurun_out/pytest_all.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
exit $rc
