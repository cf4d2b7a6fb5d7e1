#!/bin/bash
# dK / dV GEMM shapes: the current TN form (P / dS query-major) vs a key-major hand-off (NN with
# K-major A), every tile config, interleaved rounds
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
: > $OUT/dkdv.jsonl
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_gemm_step.py --only dKdV --cfg 0 1 5 11 20 30 --reps 20 >> $OUT/dkdv.jsonl 2>$OUT/dkdv.err || { tail $OUT/dkdv.err; exit 1; }
done
grep -c shape $OUT/dkdv.jsonl
