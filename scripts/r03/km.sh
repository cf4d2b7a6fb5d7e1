#!/bin/bash
# key-major P / dS hand-off (JMT_ATTN_KM=1): attention + model tests, then the c3 bench with it
# on and off, interleaved
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
JMT_ATTN_KM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/km_tests.log 2>&1
rc=$?; tail -3 $OUT/km_tests.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/km_ab.jsonl
for r in 1 2; do
  for km in 1 0; do
    JMT_ATTN_KM=$km timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline > $OUT/km_b.log 2>&1 || { tail -5 $OUT/km_b.log; exit 1; }
    python3 - $km $r >> $OUT/km_ab.jsonl <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/r03/km_b.log") if l.startswith("{")][-1]
fam = {f["family"]: [f["launches_per_step"], f["ms_per_step"], f["avg_launch_us"]] for f in d["roofline"]["families"]}
print(json.dumps({"km": int(sys.argv[1]), "round": int(sys.argv[2]), "ms_per_step": d["ms_per_step"], "parity": d["parity"]["pass"], "families": fam}))
PY
    tail -1 $OUT/km_ab.jsonl | cut -c1-250
  done
done
