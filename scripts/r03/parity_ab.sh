#!/bin/bash
# parity report with the full per-quantity dump (margins, mutation errors), then the attention
# OPT A/B (scripts/r03/attn_opt.sh)
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 900 python -u scripts/parity_report.py --dump $OUT/parity > $OUT/parity_report.jsonl 2> $OUT/parity_report.err
rc=$?; echo "report exit $rc"; cut -c1-300 $OUT/parity_report.jsonl | head -30
if [ $rc -ne 0 ]; then tail -20 $OUT/parity_report.err; exit $rc; fi
bash scripts/r03/attn_opt.sh
