#!/bin/bash
# Dev tool (GPU box): interleaved A/B of the Gym step() launch (tools/step_ab.py) over
# STEP_VARIANTS="name[@pf]..." -- libmev_<name>.so, with MEV_STEP_PF=<pf> when given; REPS rounds;
# WL / E as tools/step_ab.py. Lines go to gpurun_out/step_ab.log.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for vs in ${STEP_VARIANTS:-base}; do
    v=${vs%%@*}; pf=1; [ "$vs" != "$v" ] && pf=${vs#*@}
    MEV_STEP_PF=$pf MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_$v.so timeout -k 10 120 \
      python -u tools/step_ab.py "$vs" > gpurun_out/step_tmp.log 2>&1 \
      || { echo "variant $vs failed"; cat gpurun_out/step_tmp.log; exit 1; }
    grep '^{' gpurun_out/step_tmp.log | tee -a gpurun_out/step_ab.log
  done
done
