#!/bin/bash
# GEMM schedule experiment (cfg 6 = 128x128 + s_setprio vs the planner), forced-config kernel
# tests, the step-shape microbenchmark, then the default bench with its CPU baseline.
set -u
OUT=gpurun_out; mkdir -p $OUT
JMT_GEMM_CFG=6 timeout -k 10 200 python -m pytest tests/test_gpu_kernels.py -q -x --timeout 150 -p no:cacheprovider -k gemm > $OUT/kcfg6.log 2>&1
rc=$?; echo "cfg 6 tests: $(tail -1 $OUT/kcfg6.log)"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm_step.py --cfg 0 1 6 > $OUT/sched_step2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_prio.log 2>&1 || exit $?
tail -1 $OUT/bench_prio.log
