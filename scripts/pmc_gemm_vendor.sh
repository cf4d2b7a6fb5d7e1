#!/bin/bash
# PMC: gemm.hip vs hipBLASLt on NT b3 19200x512x512 and NN b6 19200x512x1024; bounds test -v
set -u
OUT=gpurun_out/r04/pmc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k bounds -v -s -p no:cacheprovider > gpurun_out/r04/g2_bounds.log 2>&1
echo "bounds exit $?"; grep -i "violations\|passed\|failed" gpurun_out/r04/g2_bounds.log | tail -3
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CU_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/gemm_vs_vendor.py --only "NT b3 19200x512x512,NN b6,NT b1" --reps 3 --rounds 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
      python3 scripts/gemm_vs_vendor.py --only "NT b3 19200x512x512,NN b6,NT b1" --reps 5 --rounds 1 > $OUT/kt.log 2>&1
echo "pmc done $?"
