#!/bin/bash
# grouped branches: full GPU test suite, then bench graph / eager / ungrouped
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-gr}
JMT_CAPTURE_STREAMS=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -25 $OUT/${TAG}_tests.log | grep -v "^  " | tail -12
if [ $rc -gt 1 ]; then exit $rc; fi
run() {  # name, env..., args
  local name=$1; shift
  env "$@" JMT_CAPTURE_STREAMS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/${TAG}_$name.log 2>&1
  local r=$?; echo "bench $name exit $r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"host_issue_ms_per_eager_step": [0-9.]*\|"frac": [0-9.]*' $OUT/${TAG}_$name.log | tr '\n' ' ')"
  if [ $r -ne 0 ]; then tail -20 $OUT/${TAG}_$name.log; fi
  return $r
}
run graph JMT_GROUPED=1 && BENCH_EXTRA=--no-graph run eager JMT_GROUPED=1 && BENCH_EXTRA=--no-graph run eager_ungrouped JMT_GROUPED=0
