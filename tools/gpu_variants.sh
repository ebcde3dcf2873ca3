set -o pipefail
for v in ${VARIANTS:-a0_w1}; do
  MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_$v.so MODES=${MODES:-rollout} timeout -k 10 120 python -u tools/rollout_modes.py >> gpurun_out/variants.log 2>&1 || exit 1
done
