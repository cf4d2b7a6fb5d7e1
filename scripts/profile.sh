#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no per-launch events, no CPU baseline).
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-probe ${BENCH_ARGS:-} \
    > $OUT/bench_stdout.log 2>&1
rc=$?
echo "rocprof exit $rc"
find $OUT -name "*kernel_stats.csv" | head -3
exit $rc
