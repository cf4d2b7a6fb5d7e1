#!/bin/bash
# split-K qkv / FFN1 wgrad (1536x512, b3) tile / split sweep, twice (order effects)
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_gemm_step.py --only "1536x512xR" --cfg 0 5 10 1 --splits 0 4 6 8 10 > $OUT/b8_wgrad_$r.jsonl 2>&1 || { tail -5 $OUT/b8_wgrad_$r.jsonl; exit 1; }
done
