#!/bin/bash
# GPU-box check: tests, smoke, short bench.  Stops at the first crash / timeout (not at test
# failures, which are ordinary exit 1).
set -u
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?
echo "pytest exit $rc" | tee -a $OUT/${TAG}_tests.log
tail -15 $OUT/${TAG}_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1
rc=$?
echo "smoke exit $rc"; tail -3 $OUT/${TAG}_smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > $OUT/${TAG}_bench.log 2>&1
rc=$?
echo "bench exit $rc"; tail -5 $OUT/${TAG}_bench.log
exit $rc
