#!/bin/bash
# row sums via v_dot2 (branch-free): GEMM tests, wgrad +dbias tile sweep, LN bwd 32-row blocks
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or layernorm" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/b7_kern.log 2>&1
rc=$?; tail -2 $OUT/b7_kern.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_gemm_step.py --only "wgrad" --cfg 0 1 5 10 > $OUT/b7_wgrad.jsonl 2>&1 || { tail -5 $OUT/b7_wgrad.jsonl; exit 1; }
timeout -k 10 200 python scripts/bench_rowops.py --out $OUT/rowops_b7.jsonl > $OUT/b7_rowops.log 2>&1 || { tail -5 $OUT/b7_rowops.log; exit 1; }
grep ln_bwd $OUT/rowops_b7.jsonl
: > $OUT/bgrad_ab2.jsonl
for r in 1 2; do
  for fb in 1 0; do
    JMT_FUSED_BGRAD=$fb timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > $OUT/b7_b.log 2>&1 || { tail -5 $OUT/b7_b.log; exit 1; }
    grep '^{' $OUT/b7_b.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'fused_bgrad':$fb,'round':$r,'ms_per_step':d['ms_per_step'],'parity':d.get('parity')}))" >> $OUT/bgrad_ab2.jsonl
    tail -1 $OUT/bgrad_ab2.jsonl | cut -c1-120
  done
done
