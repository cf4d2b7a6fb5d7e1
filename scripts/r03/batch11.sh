#!/bin/bash
# launch logs of the short-sequence configs (which launches a realdata / c2 step is made of)
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
for c in realdata c2; do
  timeout -k 10 200 python bench.py --config $c --steps 100 --no-cpu-baseline --launch-log $OUT/launch_$c.jsonl > $OUT/b11_$c.log 2>&1 || { tail -5 $OUT/b11_$c.log; exit 1; }
  grep '^{' $OUT/b11_$c.log | tail -1 | cut -c1-200
done
