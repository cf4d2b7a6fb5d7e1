#!/bin/bash
# GPU test suite (optionally a subset: $1 = pytest selection), log under gpurun_out/r03/
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
TAG=${TAG:-tests}
timeout -k 10 900 python -u -m pytest ${1:-tests} -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}.log 2>&1
rc=$?; echo "tests exit $rc"; tail -15 $OUT/${TAG}.log
exit $rc
