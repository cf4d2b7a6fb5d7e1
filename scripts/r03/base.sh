#!/bin/bash
# round-3 baseline: GPU tests, then the plain default bench command
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/base_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -5 $OUT/base_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/base_bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep '^{' $OUT/base_bench.log | tail -1 | cut -c1-600
exit $rc
