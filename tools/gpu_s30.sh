#!/bin/bash
# Session 30: the box's plain-store write rate (tools/write_ceiling.py) next to the headline's
# 20 / 200-step launches on the same box (tools/launch_len.py), twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/write_ceiling.py >> gpurun_out/write_ceiling.log 2>&1 || { tail -20 gpurun_out/write_ceiling.log; exit 1; }
  timeout -k 10 120 python -u tools/launch_len.py 20 200 > gpurun_out/ll_tmp.log 2>&1 || { tail -20 gpurun_out/ll_tmp.log; exit 1; }
  grep '^{' gpurun_out/ll_tmp.log >> gpurun_out/write_ceiling.log
done
cat gpurun_out/write_ceiling.log | grep '^{' | cut -c1-220
