#!/bin/bash
# persistent attention: kernel tests, A/B micro-bench, all GPU tests, short bench
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fused_attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/s3b_attn_tests.log 2>&1
rc=$?; echo "attn tests exit $rc"; tail -3 $OUT/s3b_attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 0 1; do
  JMT_ATTN_PERSIST=$m timeout -k 10 120 python scripts/bench_attn.py 384 300 20 >> $OUT/s3b_attn_bench.log 2>&1 || exit 1
  JMT_ATTN_PERSIST=$m timeout -k 10 120 python scripts/bench_attn.py 192 300 20 >> $OUT/s3b_attn_bench.log 2>&1 || exit 1
  JMT_ATTN_PERSIST=$m timeout -k 10 120 python scripts/bench_attn.py 96 1024 10 >> $OUT/s3b_attn_bench.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/s3b_attn_bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/s3b_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/s3b_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > $OUT/s3b_bench.log 2>&1
rc=$?; echo "bench exit $rc"; grep -o '"ms_per_step": [0-9.]*\|"family": "[a-z_A-Z]*"\|"frac": [0-9.]*' $OUT/s3b_bench.log | tr '\n' ' '
exit $rc
