#!/bin/bash
set -u
OUT=gpurun_out/prof_evt; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/event_check.py > $OUT/plain.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
    python3 scripts/event_check.py > $OUT/prof.log 2>&1 || exit $?
grep per_launch $OUT/plain.log; grep per_launch $OUT/prof.log
