#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass; counters only with --kernel-trace) on a command.
#   bash scripts/pmc.sh TAG -- python3 scripts/bench_gemm.py --only NT --reps 5
set -u
TAG=$1; shift; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/p$i -o run -- "$@" \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc done"
