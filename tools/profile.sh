#!/bin/bash
# rocprofv3 profile of bench.py's launches (run on the GPU box from the repo root):
#   1. --kernel-trace --stats              -> per-kernel average duration
#   2. --pmc FETCH_SIZE                    (own pass)
#   3. --pmc WRITE_SIZE                    (own pass)
#   4. --pmc SQ_* occupancy/issue counters (own pass)
#   5. --pmc SQ_INSTS_* / GRBM              (own pass)
#   6. --pmc SQ LDS counters                 (own pass)
# Counters run in separate passes with --kernel-trace only (no sys/runtime tracing). The raw
# rocprofv3 output stays in box-local scratch (/tmp); tools/pmc_summary.py writes the summary to
# gpurun_out/profiles/ (copied back), which tools/merge_profiles.py folds into profiles/.
# usage: tools/profile.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r02}; shift
ARGS="--profile-run --steps 1000 --warmup 1001 --warmup-floor-s 2 $*"
RAW=/tmp/prof_$TAG
OUT=gpurun_out/profiles
mkdir -p $RAW $OUT
export TMPDIR=/tmp
run() {  # name, extra rocprof args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $RAW/$name -o $name --output-format csv -- python3 bench.py $ARGS > $RAW/$name.log 2>&1 \
    || { echo "rocprofv3 $name failed"; tail -20 $RAW/$name.log; return 1; }
}
run kt --kernel-trace --stats &&
run fetch --kernel-trace --pmc FETCH_SIZE &&
run write --kernel-trace --pmc WRITE_SIZE &&
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run sq2 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD &&
run sq3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU &&
python3 tools/pmc_summary.py $RAW $TAG "$ARGS" $OUT > $OUT/${TAG}_summary.log 2>&1 &&
echo "profile done: $OUT/${TAG}_pmc.json"
