#!/bin/bash
# Session 26: the driver's two bench command lines on the final tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_s26_driver.json 2> gpurun_out/bench_s26_driver.err || { tail -20 gpurun_out/bench_s26_driver.err; exit 1; }
tail -c 300 gpurun_out/bench_s26_driver.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_s26.json 2> gpurun_out/bench_s26.err || { tail -20 gpurun_out/bench_s26.err; exit 1; }
tail -c 300 gpurun_out/bench_s26.json
