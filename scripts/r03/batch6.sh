#!/bin/bash
# bias gradients as A row sums of the weight-gradient GEMM: kernel + model tests, GEMM shapes,
# c3 A/B (JMT_FUSED_BGRAD)
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/b6_kern.log 2>&1
rc=$?; tail -2 $OUT/b6_kern.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_gpu_train.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/b6_tests.log 2>&1
rc=$?; tail -2 $OUT/b6_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/bench_gemm_step.py --only wgrad > $OUT/b6_wgrad.jsonl 2>&1 || { tail -5 $OUT/b6_wgrad.jsonl; exit 1; }
: > $OUT/bgrad_ab.jsonl
for r in 1 2; do
  for fb in 1 0; do
    JMT_FUSED_BGRAD=$fb timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > $OUT/b6_b.log 2>&1 || { tail -5 $OUT/b6_b.log; exit 1; }
    grep '^{' $OUT/b6_b.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'fused_bgrad':$fb,'round':$r,'ms_per_step':d['ms_per_step'],'parity':d.get('parity')}))" >> $OUT/bgrad_ab.jsonl
    tail -1 $OUT/bgrad_ab.jsonl | cut -c1-200
  done
done
