#!/bin/bash
# A/B of the attention kernels' OPT bits (JMT_ATTN_OPT): kernel tests under OPT=7, then
# bench_attn.py at the c3 cross-attention (384 x 300) and encoder (192 x 300) launches, arms
# interleaved over two rounds
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
JMT_ATTN_OPT=7 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "attention or attn" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/attn_opt_tests.log 2>&1
rc=$?; tail -2 $OUT/attn_opt_tests.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/attn_opt.jsonl
for round in 1 2; do
  for o in ${OPTS:-0 1 2 4 8 16 7 15 31}; do
    for shape in "384 300 40" "192 300 40"; do
      r=$(JMT_ATTN_OPT=$o timeout -k 10 120 python scripts/bench_attn.py $shape) || exit 1
      echo "{\"opt\": $o, \"round\": $round, \"r\": $r}" | tee -a $OUT/attn_opt.jsonl
    done
  done
done
