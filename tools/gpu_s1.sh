set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --maxfail=10 --timeout 150 --timeout-method thread > gpurun_out/pytest_s1.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_s1.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_s1_driver.json 2> gpurun_out/bench_s1_driver.err || exit 1
tail -c 1500 gpurun_out/bench_s1_driver.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_s1.json 2> gpurun_out/bench_s1.err || exit 1
tail -c 600 gpurun_out/bench_s1.json
