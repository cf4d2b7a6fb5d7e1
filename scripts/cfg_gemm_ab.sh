#!/bin/bash
set -u
OUT=gpurun_out/r05; mkdir -p $OUT
for c in realdata c4; do
  for v in "0 0" "40 1" "0 1" "40 0"; do
    set -- $v
    if [ $1 = 0 ]; then unset JMT_GEMM_PERSIST; else export JMT_GEMM_PERSIST=$1; fi
    export JMT_GEMM_PPSPLIT=$2
    timeout -k 10 200 python3 bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-parity > $OUT/cab_${c}_$1_$2.log 2>&1 || exit 1
    echo "$c persist=$1 ppsplit=$2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/cab_${c}_$1_$2.log | head -1)" >> $OUT/cab.txt
  done
done
