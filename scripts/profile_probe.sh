#!/bin/bash
# rocprofv3 kernel trace of the default bench WITH its per-launch HIP-event probe, so the probe's
# average NT-GEMM launch time and rocprof's durations of the same launches come from one run.
set -u
TAG=${1:-r01p}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_stdout.log 2>&1
rc=$?; echo "rocprof exit $rc"; tail -1 $OUT/bench_stdout.log | grep -o '"avg_launch_us": [0-9.]*'
exit $rc
