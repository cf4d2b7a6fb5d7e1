#!/bin/bash
# pipelined attention forward: kernel tests, A/B micro-bench, all GPU tests, bench A/B
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "fused_attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pipe_attn_tests.log 2>&1
rc=$?; echo "attn tests exit $rc"; tail -3 $OUT/pipe_attn_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" $OUT/pipe_attn_tests.log | head; exit $rc; fi
rm -f $OUT/pipe_attn_bench.log
for m in 0 1; do
  JMT_ATTN_PIPE=$m timeout -k 10 120 python scripts/bench_attn.py 384 300 20 >> $OUT/pipe_attn_bench.log 2>&1 || exit 1
  JMT_ATTN_PIPE=$m timeout -k 10 120 python scripts/bench_attn.py 192 300 20 >> $OUT/pipe_attn_bench.log 2>&1 || exit 1
  JMT_ATTN_PIPE=$m timeout -k 10 120 python scripts/bench_attn.py 96 1024 10 >> $OUT/pipe_attn_bench.log 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/pipe_attn_bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pipe_tests.log 2>&1
rc=$?; echo "tests exit $rc"; tail -3 $OUT/pipe_tests.log
if [ $rc -gt 1 ]; then grep -E "FAIL|Error" $OUT/pipe_tests.log | head; exit $rc; fi
for m in 0 1 0 1; do
  JMT_ATTN_PIPE=$m timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --probe-steps 1 > $OUT/pipe_bench_$m.log 2>&1 || exit 1
  echo "pipe=$m $(grep -o '"ms_per_step": [0-9.]*' $OUT/pipe_bench_$m.log | head -1)"
done
