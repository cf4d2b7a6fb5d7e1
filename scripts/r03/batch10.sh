#!/bin/bash
# final build: whole GPU suite + default bench (the driver's round-end commands)
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/b10_tests.log 2>&1
rc=$?; tail -3 $OUT/b10_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/b10_smoke.log 2>&1 || { tail -5 $OUT/b10_smoke.log; exit 1; }
tail -1 $OUT/b10_smoke.log
timeout -k 10 400 python bench.py > $OUT/b10_bench.log 2>&1 || { tail -5 $OUT/b10_bench.log; exit 1; }
grep '^{' $OUT/b10_bench.log | tail -1 | cut -c1-400
for u in 2 4; do
  JMT_LN_BWD_U=$u timeout -k 10 200 python scripts/bench_rowops.py --out $OUT/rowops_u$u.jsonl > $OUT/b10_rowops.log 2>&1 || { tail -5 $OUT/b10_rowops.log; exit 1; }
  grep "ln_bwd_dsum grouped" $OUT/rowops_u$u.jsonl
done
: > $OUT/ln_u_ab.jsonl
for r in 1 2; do
  for u in 4 2; do
    JMT_LN_BWD_U=$u timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > $OUT/b10_b.log 2>&1 || { tail -5 $OUT/b10_b.log; exit 1; }
    grep '^{' $OUT/b10_b.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'ln_bwd_u':$u,'round':$r,'ms_per_step':d['ms_per_step']}))" >> $OUT/ln_u_ab.jsonl
    tail -1 $OUT/ln_u_ab.jsonl
  done
done
