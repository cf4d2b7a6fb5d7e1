#!/bin/bash
# short-sequence attention: kernel tests, the model-level tests on the shapes that now use it
# (c2 batch-axis attention, T=16 real data), then c2 / realdata benches with the short kernels
# on and off (JMT_ATTN_SHORT), interleaved
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn_short.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/short_tests.log 2>&1
rc=$?; tail -3 $OUT/short_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_realdata.py tests/test_gpu_configs.py tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/short_model_tests.log 2>&1
rc=$?; tail -3 $OUT/short_model_tests.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/short_ab.jsonl
for round in 1 2; do
  for s in 1 0; do
    for cfg in c2 realdata; do
      JMT_ATTN_SHORT=$s timeout -k 10 200 python bench.py --config $cfg --steps 100 --no-cpu-baseline > $OUT/short_b.log 2>&1 || { tail -5 $OUT/short_b.log; exit 1; }
      python3 - $s $cfg $round >> $OUT/short_ab.jsonl <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/r03/short_b.log") if l.startswith("{")][-1]
fam = {f["family"]: [f["launches_per_step"], f["ms_per_step"]] for f in (d["roofline"] or {}).get("families", [])}
print(json.dumps({"short": int(sys.argv[1]), "config": sys.argv[2], "round": int(sys.argv[3]), "ms_per_step": d["ms_per_step"], "value": d["value"], "step_mfma": d["step_mfma"], "parity": d["parity"]["pass"], "families": fam}))
PY
      tail -1 $OUT/short_ab.jsonl | cut -c1-200
    done
  done
done
