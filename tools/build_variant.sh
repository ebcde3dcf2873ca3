#!/bin/bash
# Dev tool: build libmev_<name>.so from mev_step.hip at git revision <rev> ("WT" = working tree)
# with the Makefile's flags (plus $EXTRA, e.g. -DMEV_LDS2_WAVES=8), for interleaved timing with tools/gpu_variants.sh
# or any tool run with MEV_LIB=$PWD/mobile-env-gan_amd/lib/libmev_<name>.so (tools/launch_len.py, tools/ts_probe.py).
set -e
rev=$1; name=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
src=/tmp/mev_variant_$name.hip
if [ "$rev" = WT ]; then cp "$ROOT/mobile-env-gan_amd/csrc/mev_step.hip" $src
else git -C "$ROOT" show "$rev:mobile-env-gan_amd/csrc/mev_step.hip" > $src; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall \
  -I"$ROOT/include" -mllvm -amdgpu-sched-strategy=max-ilp $EXTRA -shared -o \
  "$ROOT/mobile-env-gan_amd/lib/libmev_$name.so" $src
