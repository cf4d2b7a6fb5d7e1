#!/bin/bash
# attention kernel tests, then a short profiled c3 bench (kernel stats per step)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "attention" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1
rc=$?
tail -3 gpurun_out/attn_tests.log
[ $rc -ne 0 ] && exit $rc
STEPS=10 bash scripts/profile.sh ${1:-r02_attn} > gpurun_out/prof_${1:-r02_attn}.txt 2>&1
rc=$?
f=$(find gpurun_out/prof_${1:-r02_attn} -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 scripts/kstats.py $f 13 30 > gpurun_out/kstats_${1:-r02_attn}.txt
tail -2 gpurun_out/prof_${1:-r02_attn}/bench_stdout.log
exit $rc
