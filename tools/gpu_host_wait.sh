#!/bin/bash
# Dev tool (GPU box): the driver's bench shape (--steps 20 --warmup 5) under each HIP host wait
# policy, interleaved; one JSON line per run into gpurun_out/host_wait.jsonl.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/host_wait.jsonl
for rep in $(seq 1 ${REPS:-3}); do
  for hw in auto spin block; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-wait $hw \
      --timed-repeats 20 --step-launches 0 > gpurun_out/hw_tmp.log 2>&1 || { echo "host-wait $hw failed"; tail -20 gpurun_out/hw_tmp.log; exit 1; }
    grep '^{' gpurun_out/hw_tmp.log | tail -1 >> gpurun_out/host_wait.jsonl
    echo "rep $rep $hw done"
  done
done
