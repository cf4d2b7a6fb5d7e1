#!/bin/bash
# V / A regressor pair (input gradients summed by the autograd-rounding add): pair tests, the
# full GPU suite, bench A/B
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pair3_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/pair3_tests.log; grep -E "^FAILED|Error" $OUT/pair3_tests.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
for m in 0 1 0 1 0 1; do
  JMT_PAIR_MLP=$m timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --probe-steps 1 > $OUT/pair3_bench_$m.log 2>&1 || exit 1
  echo "pair=$m $(grep -o '"ms_per_step": [0-9.]*' $OUT/pair3_bench_$m.log | head -1)"
done
