#!/bin/bash
# Round-4 GPU session C (host side of the driver's timed region): isolated 20-step launches'
# wall time with the default HIP wait policy vs spin-wait (hipDeviceScheduleSpin = 1) and
# blocking sync (4), no events (EVMODE=none), interleaved twice.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for sp in "" 1 4; do
    SPIN=$sp EVMODE=none timeout -k 10 120 python -u tools/launch_len.py 20 > gpurun_out/spin_tmp.log 2>&1 \
      || { echo "spin $sp failed"; cat gpurun_out/spin_tmp.log; exit 1; }
    grep '^{' gpurun_out/spin_tmp.log | tee -a gpurun_out/spin.log
  done
done
# the driver's own command line, default vs spin-wait host policy, interleaved
for rep in 1 2 3; do
  for hw in auto spin; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --step-launches 0 \
      --host-wait $hw > gpurun_out/bench_hw_tmp.json 2> gpurun_out/bench_hw_tmp.err \
      || { echo "bench $hw failed"; tail -20 gpurun_out/bench_hw_tmp.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bench_hw_tmp.json'));print(json.dumps({'hw':'$hw','rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step'],'launch_ms':d['roofline']['launch_ms']}))" | tee -a gpurun_out/bench_hw.log
  done
done
