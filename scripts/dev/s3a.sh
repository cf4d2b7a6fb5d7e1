#!/bin/bash
# GPU tests + short bench + an eager-step kernel trace (ordered dispatches of one step)
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/s3a_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -5 $OUT/s3a_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/s3a_bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -c 600 $OUT/s3a_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/s3a_trace -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-graph --no-cpu-baseline --no-probe --no-parity > $OUT/s3a_trace.log 2>&1
rc=$?; echo "trace exit $rc"; exit $rc
