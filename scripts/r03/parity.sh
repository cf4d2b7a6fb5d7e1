#!/bin/bash
# round-3 parity: the per-quantity report (margins), then the GPU test suite
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 600 python -u scripts/parity_report.py > $OUT/parity_report.jsonl 2> $OUT/parity_report.err
rc=$?; echo "report exit $rc"; cut -c1-400 $OUT/parity_report.jsonl | head -12
if [ $rc -ne 0 ]; then tail -20 $OUT/parity_report.err; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/${TAG:-tests}.log 2>&1
rc=$?; echo "tests exit $rc"; grep -E "passed|failed|FAILED|Error" $OUT/${TAG:-tests}.log | tail -30
exit $rc
