#!/bin/bash
# c2-sized (9,600-row) GEMM shapes: tile configs
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 500 python scripts/bench_gemm_step.py --rows 9600 --cfg 0 1 5 11 20 30 > $OUT/b13_c2_gemm.jsonl 2>&1 || { tail -5 $OUT/b13_c2_gemm.jsonl; exit 1; }
wc -l $OUT/b13_c2_gemm.jsonl
