set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for m in auto spin yield block; do
  timeout -k 10 120 python -u tools/host_wait_probe.py $m 2 >> gpurun_out/host_wait.log 2>&1 || exit 1
done; done
grep '^{' gpurun_out/host_wait.log
