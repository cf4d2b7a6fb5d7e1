#!/bin/bash
# grouped wo_JR (c2): model / config / 2-rank tests, then c2 with the grouped path on and off
set -u
OUT=gpurun_out/r03; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $OUT/b4_tests.log 2>&1
rc=$?; tail -2 $OUT/b4_tests.log; [ $rc -ne 0 ] && exit $rc
: > $OUT/c2_grouped_ab.jsonl
for r in 1 2; do
  for gr in 1 0; do
    JMT_GROUPED=$gr timeout -k 10 200 python bench.py --config c2 --steps 100 --no-cpu-baseline > $OUT/b4_b.log 2>&1 || { tail -5 $OUT/b4_b.log; exit 1; }
    python3 - $gr $r >> $OUT/c2_grouped_ab.jsonl <<'PY'
import json, sys
d = [json.loads(l) for l in open("gpurun_out/r03/b4_b.log") if l.startswith("{")][-1]
fam = {f["family"]: [f["launches_per_step"], f["ms_per_step"]] for f in d["roofline"]["families"]}
print(json.dumps({"grouped": int(sys.argv[1]), "round": int(sys.argv[2]), "ms_per_step": d["ms_per_step"], "step_mfma": d["step_mfma"]["frac_of_peak"], "parity": d["parity"], "families": fam}))
PY
    tail -1 $OUT/c2_grouped_ab.jsonl | cut -c1-160
  done
done
timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > $OUT/b4_c3.log 2>&1 || { tail -5 $OUT/b4_c3.log; exit 1; }
grep '^{' $OUT/b4_c3.log | cut -c1-400
