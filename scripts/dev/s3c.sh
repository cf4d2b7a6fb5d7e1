#!/bin/bash
# new dK/dV tile configs: forced-config kernel tests, step-shape sweep on the dK/dV shape
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "forced_configs" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/s3c_tests.log 2>&1
rc=$?; echo "cfg tests exit $rc"; tail -3 $OUT/s3c_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_gemm_step.py --cfg 0 11 22 23 1 10 --only dKdV --reps 30 > $OUT/s3c_sweep.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/s3c_sweep.log; exit $rc
