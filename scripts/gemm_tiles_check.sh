#!/bin/bash
# GEMM tile-config sweep on the GPU box: parity tests per forced config, then the microbench.
#   bash scripts/gemm_tiles_check.sh "5 8 9" "1 5 8 9"
set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
TEST_CFGS=${1:-"0 5"}
BENCH_CFGS=${2:-"1 5 0"}
for c in $TEST_CFGS; do
  JMT_GEMM_CFG=$c timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q -k gemm -p no:cacheprovider > gpurun_out/gemm_test_cfg$c.log 2>&1 || { echo "cfg $c FAILED"; tail -30 gpurun_out/gemm_test_cfg$c.log; exit 1; }
  echo "cfg $c: $(tail -1 gpurun_out/gemm_test_cfg$c.log)"
done
timeout -k 10 400 python scripts/bench_gemm.py --cfg $BENCH_CFGS > gpurun_out/bench_gemm_tiles.log 2>&1
python - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/bench_gemm_tiles.log") if l.startswith("{")]
t = collections.defaultdict(dict)
for r in rows:
    t[r["shape"]][r["cfg"]] = r["us"]
cfgs = sorted({r["cfg"] for r in rows})
print("shape".ljust(34) + "".join(f"{c:>9}" for c in cfgs))
for s, d in t.items():
    print(s.ljust(34) + "".join(f"{d.get(c, 0):9.1f}" for c in cfgs))
PY
