#!/bin/bash
# B*T-row overrides keyed to >= 16,384 rows: c2 / c3 / realdata benches, GEMM kernel tests
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/b14_kern.log 2>&1
rc=$?; tail -2 $OUT/b14_kern.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/b14_bench.jsonl
for c in c2 c3 c2 c3 realdata; do
  timeout -k 10 200 python bench.py --config $c --steps 200 --no-cpu-baseline > $OUT/b14_b.log 2>&1 || { tail -5 $OUT/b14_b.log; exit 1; }
  grep '^{' $OUT/b14_b.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config':'$c','ms_per_step':d['ms_per_step'],'value':d['value'],'step_mfma':d.get('step_mfma',{}).get('frac_of_peak')}))" >> $OUT/b14_bench.jsonl
  tail -1 $OUT/b14_bench.jsonl
done
timeout -k 10 500 python scripts/bench_gemm_step.py --rows 9600 --cfg 0 > $OUT/b14_c2_gemm.jsonl 2>&1 || { tail -5 $OUT/b14_c2_gemm.jsonl; exit 1; }
