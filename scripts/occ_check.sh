#!/bin/bash
# GEMM occupancy experiment (cfg 10/11: 128x128 KB64 at 4/3 blocks per CU) vs the planner and
# cfg 1: forced-config kernel tests, the step-shape microbenchmark, then smoke().
set -u
OUT=gpurun_out; mkdir -p $OUT
for c in 10 11; do
  JMT_GEMM_CFG=$c timeout -k 10 200 python -m pytest tests/test_gpu_kernels.py -q -x --timeout 150 -p no:cacheprovider -k gemm > $OUT/kcfg$c.log 2>&1
  rc=$?; echo "cfg $c tests: $(tail -1 $OUT/kcfg$c.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 300 python scripts/bench_gemm_step.py --cfg 1 0 10 11 > $OUT/occ_step.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke exit $?"; tail -1 $OUT/smoke.log
