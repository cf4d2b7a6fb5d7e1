#!/bin/bash
# GPU-box round: all GPU tests, then the default bench and a rocprofv3 kernel-trace profile.
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-rr}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -25 $OUT/${TAG}_tests.log | grep -v "^  " | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:---no-cpu-baseline} > $OUT/${TAG}_bench.log 2>&1
rc=$?; echo "bench exit $rc: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"achieved": [0-9.]*\|"avg_launch_us": [0-9.]*' $OUT/${TAG}_bench.log | tr '\n' ' ')"
if [ $rc -ne 0 ]; then tail -20 $OUT/${TAG}_bench.log; exit $rc; fi
if [ -n "${PROFILE:-}" ]; then bash scripts/profile.sh $TAG; fi
