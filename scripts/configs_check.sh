#!/bin/bash
# other BASELINE.json workloads (parity / profiling cases) + real-data shape path test
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-cfg}
timeout -k 5 200 python -u -m pytest tests/test_gpu_realdata.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_realdata.log 2>&1
rc=$?; echo "realdata tests exit $rc"; tail -3 $OUT/${TAG}_realdata.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in ${CONFIGS:-realdata c2 c4 c5 c3sa}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/${TAG}_$c.log 2>&1
  r=$?; echo "$c exit $r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac_of_peak": [0-9.]*' $OUT/${TAG}_$c.log | tr '\n' ' ')"
  if [ $r -ne 0 ]; then tail -12 $OUT/${TAG}_$c.log; exit $r; fi
done
