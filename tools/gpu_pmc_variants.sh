# PMC passes of the rollout launch for library variants (dev tool; run on the GPU box):
#   VARIANTS="base w8" bash tools/gpu_pmc_variants.sh
set -o pipefail
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
for v in ${VARIANTS:-base}; do
  for pass in A B; do
    C=${!pass}
    MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_$v.so MODES=${MODES:-rollout} K=2000 \
      timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmcv/$v$pass -o p --output-format csv \
      -- python3 tools/rollout_modes.py > gpurun_out/pmcv_$v$pass.log 2>&1 || { tail -5 gpurun_out/pmcv_$v$pass.log; exit 1; }
  done
done
