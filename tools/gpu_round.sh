#!/bin/bash
# One GPU session (run from the repo root on the box): STEPS selects the parts, in order --
#   tests  pytest -m gpu (PYTEST_ARGS, limit PYTEST_LIMIT s) + smoke()
#   ab     interleaved A/B of libmev_<v>.so variants (VARIANTS, REPS, LENS, WL; tools/ab.sh)
#   abm    the same at 4,096 medium envs (MVARIANTS, MLENS)
#   ts     per-wave phase stamps of one TS_LEN-step launch (libmev_ts.so, tools/ts_probe.py)
#   prof   committed-profile passes (tools/profile.sh) for PROF="tag:args;tag:args"
#   bench  bench.py lines: the driver's shape (--steps 20 --warmup 5) and the default run
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in ${STEPS:-tests}; do
  case $s in
  tests)
    timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -x -v -m gpu --timeout 150 \
      --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
      || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
    tail -3 gpurun_out/pytest_gpu.log
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
    tail -1 gpurun_out/smoke.log ;;
  ab)
    rm -f gpurun_out/ab.log
    bash tools/ab.sh || exit 1 ;;
  abm)  # medium @ 4,096 (BASELINE configs[1]), appended to the same log
    WL=mobile-medium-central-v0 E=4096 VARIANTS="${MVARIANTS:-base new}" LENS="${MLENS:-200}" \
      bash tools/ab.sh || exit 1 ;;
  ts)
    MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=${TS_REPS:-3} timeout -k 10 120 \
      python tools/ts_probe.py ${TS_LEN:-20} > gpurun_out/ts.log 2>&1 || { echo ts failed; tail gpurun_out/ts.log; exit 1; }
    tail -5 gpurun_out/ts.log ;;
  prof)
    IFS=';' read -ra P <<< "$PROF"
    for pa in "${P[@]}"; do
      tag=${pa%%:*}; args=${pa#*:}; [ "$args" = "$pa" ] && args=""
      bash tools/profile.sh $tag $args || exit 1
    done ;;
  bench)
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json \
      2> gpurun_out/bench_driver.err || { echo bench driver failed; tail gpurun_out/bench_driver.err; exit 1; }
    tail -c 300 gpurun_out/bench_driver.json
    timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
      || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
    tail -c 300 gpurun_out/bench.json ;;
  esac
done
echo session done
