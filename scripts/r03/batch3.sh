#!/bin/bash
# head reduce + b2 dgrad tile: kernel / pair / model tests, the default bench, then per-launch logs
# of the c2 and realdata workloads
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp_pair.py tests/test_gpu_models.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/b3_tests.log 2>&1
rc=$?; tail -2 $OUT/b3_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b3_bench.log 2>&1 || { tail -5 $OUT/b3_bench.log; exit 1; }
grep '^{' $OUT/b3_bench.log | tail -1 | cut -c1-220
for cfg in c2 realdata; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --launch-log $OUT/${cfg}_launch.jsonl > $OUT/b3_$cfg.log 2>&1 || { tail -5 $OUT/b3_$cfg.log; exit 1; }
  grep '^{' $OUT/b3_$cfg.log | tail -1 | cut -c1-200
done
