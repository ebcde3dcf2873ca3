#!/bin/bash
# Dev tool (GPU box): interleaved A/B of libmev variants (tools/build_variant.sh) on one box.
#   VARIANTS="base nt sc1" REPS=3 LENS="20 200" bash tools/ab.sh
# Each (rep, variant) runs tools/launch_len.py with MEV_LIB pointing at libmev_<variant>.so;
# lines go to gpurun_out/ab.log tagged with the variant. The first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for vs in ${VARIANTS:-base}; do
    v=${vs%%@*}; eo=""; [ "$vs" != "$v" ] && eo=${vs#*@}  # name[@key=v,key=v]: engine overrides
    MEV_ENGINE=$eo MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_$v.so timeout -k 10 120 python -u tools/launch_len.py ${LENS:-20 200} \
      > gpurun_out/ab_tmp.log 2>&1 || { echo "variant $v failed"; cat gpurun_out/ab_tmp.log; exit 1; }
    grep '^{' gpurun_out/ab_tmp.log | sed "s/^{/{\"variant\": \"$vs\", \"wl\": \"${WL:-large}\", \"rep\": $rep, /" | tee -a gpurun_out/ab.log
  done
done
