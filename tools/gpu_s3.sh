#!/bin/bash
# Round-4 GPU session 3: GPU tests on the tile-flush kernel, per-wave phase stamps of the
# driver's 20-step launch, and the driver's command line under the default vs spin host wait.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/pytest_s3.log 2>&1 || { tail -30 gpurun_out/pytest_s3.log; exit 1; }
tail -2 gpurun_out/pytest_s3.log
RAW=gpurun_out/ts_raw20.npy MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_ts.so REPS=4 timeout -k 10 150 python -u tools/ts_probe.py 20 200 > gpurun_out/ts_s3.log 2>&1 || { tail gpurun_out/ts_s3.log; exit 1; }
for rep in 1 2 3; do
  for hw in auto spin; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --step-launches 0 \
      --host-wait $hw > gpurun_out/bench_hw_tmp.json 2> gpurun_out/bench_hw_tmp.err \
      || { echo "bench $hw failed"; tail -20 gpurun_out/bench_hw_tmp.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_hw_tmp.json'));print(json.dumps({'hw':'$hw','rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step'],'launch_ms':d['roofline']['launch_ms']}))" | tee -a gpurun_out/bench_hw.log
  done
done
