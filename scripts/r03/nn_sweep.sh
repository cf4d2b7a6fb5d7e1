#!/bin/bash
# dgrad (NN) step shapes under every tile config, two interleaved rounds
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
: > $OUT/nn_sweep.jsonl
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_gemm_step.py --only "dgrad NN" --cfg 0 1 5 11 20 30 --reps 20 >> $OUT/nn_sweep.jsonl 2>$OUT/nn_sweep.err || { tail $OUT/nn_sweep.err; exit 1; }
done
grep -c shape $OUT/nn_sweep.jsonl
