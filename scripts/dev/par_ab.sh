#!/bin/bash
# stream-gradient GEMMs of the cross-attention backward on branch streams: GPU tests, bench A/B
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/par_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/par_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/par_tests.log | head; exit $rc; fi
for m in 0 1 0 1 0 1; do
  JMT_PAR_STREAM_DGRAD=$m timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --probe-steps 1 > $OUT/par_bench_$m.log 2>&1 || exit 1
  echo "par=$m $(grep -o '"ms_per_step": [0-9.]*' $OUT/par_bench_$m.log | head -1)"
done
