#!/bin/bash
set -u
for c in 1 2 3 4; do
  JMT_GEMM_CFG=$c timeout -k 10 200 python -m pytest tests/test_gpu_kernels.py -q -x --timeout 150 -p no:cacheprovider -k gemm > gpurun_out/kcfg$c.log 2>&1
  echo "cfg $c: $(tail -1 gpurun_out/kcfg$c.log)"
done
timeout -k 10 300 python scripts/bench_gemm.py --cfg 1 2 3 4 > gpurun_out/gemm_cfg.log 2>&1
echo bench exit $?
