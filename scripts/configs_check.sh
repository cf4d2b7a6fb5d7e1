#!/bin/bash
# other BASELINE.json workloads (parity / profiling cases) + real-data shape path test.
# Each workload's bench line is parsed as JSON (round 5's grep of "[0-9.]*" cut exponents:
# c5's parity 8.82e-05 read as 8.82).
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-cfg}
timeout -k 5 200 python -u -m pytest tests/test_gpu_realdata.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_realdata.log 2>&1
rc=$?; echo "realdata tests exit $rc"; tail -1 $OUT/${TAG}_realdata.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in ${CONFIGS:-realdata c2 c4 c5 c3sa}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > $OUT/${TAG}_$c.log 2>&1
  r=$?
  if [ $r -ne 0 ]; then echo "$c exit $r"; tail -12 $OUT/${TAG}_$c.log; exit $r; fi
  tail -1 $OUT/${TAG}_$c.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
p = d.get('parity') or {}
ns = [v for k, v in p.items() if k.startswith('north_star')]
fam = ', '.join(f\"{f['family']} {f['ms_per_step']:.3f}\" for f in (d.get('roofline') or {}).get('families', [])[:6])
print(f\"$c: {d['ms_per_step']} ms/step, {d['value']} windows/s, step_mfma {(d.get('step_mfma') or {}).get('frac_of_peak')}, \"
      f\"parity pred_max_abs_err {p.get('pred_max_abs_err')!r} (tolerance {p.get('tolerance')}, pass {p.get('pass')}), \"
      f\"north_star {ns[0]['verdict'] if ns else None}; families (ms/step): {fam}\")"
done
