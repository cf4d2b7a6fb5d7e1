#!/bin/bash
# realdata (1024-row) GEMM shapes: planner split-K vs forced splits, 128x128 vs 256x256
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 400 python scripts/bench_gemm_step.py --rows 1024 --cfg 0 1 --splits 0 1 2 4 8 > $OUT/b12_rd_gemm.jsonl 2>&1 || { tail -5 $OUT/b12_rd_gemm.jsonl; exit 1; }
wc -l $OUT/b12_rd_gemm.jsonl
timeout -k 10 500 python scripts/bench_gemm_step.py --rows 9600 --cfg 0 1 5 11 20 30 > $OUT/b13_c2_gemm.jsonl 2>&1 || { tail -5 $OUT/b13_c2_gemm.jsonl; exit 1; }
wc -l $OUT/b13_c2_gemm.jsonl
