#!/bin/bash
# Dev GPU call: all GPU tests (optionally -k $K), smoke, then bench lines ("ARGS|ARGS|...") and,
# with PROF="TAG:ARGS;TAG:ARGS", rocprofv3 profiles (tools/profile.sh) -- each under its own
# time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu ${K:+-k "$K"} --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
IFS='|' read -ra BENCHES <<< "$1"
i=0
for b in "${BENCHES[@]}"; do
  envs=""; args="$b"
  if [[ "$b" == *"::"* ]]; then envs="${b%%::*}"; args="${b#*::}"; fi  # "VAR=x VAR2=y::ARGS"
  timeout -k 10 300 env $envs python bench.py $args > gpurun_out/bench_$i.log 2>&1 || { echo "bench $b failed"; tail -30 gpurun_out/bench_$i.log; exit 1; }
  echo "== $b"; tail -1 gpurun_out/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value %.4g ms/step %.4f launch_ms %.4f frac %.3f canon %.3f' % (d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], r['canonical_equiv_frac']), 'step_roof', d['roofline_step'] and round(d['roofline_step']['launch_ms'],4))"
  i=$((i+1))
done
if [ -n "$PROF" ]; then
  IFS=';' read -ra PS <<< "$PROF"
  for p in "${PS[@]}"; do
    tools/profile.sh ${p%%:*} ${p#*:} || exit 1
  done
  python tools/merge_profiles.py > /dev/null || exit 1
fi
