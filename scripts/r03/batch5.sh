#!/bin/bash
# row-kernel micro-benchmark; other configs on the grouped-LN build
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 200 python scripts/bench_rowops.py --out $OUT/rowops.jsonl > $OUT/b5_rowops.log 2>&1 || { tail -5 $OUT/b5_rowops.log; exit 1; }
: > $OUT/other_configs.jsonl
for c in c2 realdata c3sa c4 c5; do
  timeout -k 10 240 python bench.py --config $c --steps 50 --no-cpu-baseline > $OUT/b5_$c.log 2>&1 || { tail -5 $OUT/b5_$c.log; exit 1; }
  grep '^{' $OUT/b5_$c.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'config':'$c','ms_per_step':d['ms_per_step'],'value':d['value'],'step_mfma':d.get('step_mfma',{}).get('frac_of_peak')}))" >> $OUT/other_configs.jsonl
  tail -1 $OUT/other_configs.jsonl
done
