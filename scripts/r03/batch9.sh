#!/bin/bash
# bias row sums also for the K-concatenated / MLP-pair wgrads: tests, c3 / c2 / realdata benches,
# qkv-wgrad tile / split sweep
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/b9_kern.log 2>&1
rc=$?; tail -2 $OUT/b9_kern.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_train.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/b9_tests.log 2>&1
rc=$?; tail -2 $OUT/b9_tests.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/b9_bench.jsonl
for c in c3 c3 c2 realdata; do
  timeout -k 10 200 python bench.py --config $c --steps 200 --no-cpu-baseline > $OUT/b9_b.log 2>&1 || { tail -5 $OUT/b9_b.log; exit 1; }
  grep '^{' $OUT/b9_b.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config':'$c','ms_per_step':d['ms_per_step'],'value':d['value']}))" >> $OUT/b9_bench.jsonl
  tail -1 $OUT/b9_bench.jsonl
done
timeout -k 10 200 python scripts/bench_gemm_step.py --only "1536x512xR" --cfg 0 5 10 1 --splits 0 4 7 10 > $OUT/b9_wgrad.jsonl 2>&1 || { tail -5 $OUT/b9_wgrad.jsonl; exit 1; }
