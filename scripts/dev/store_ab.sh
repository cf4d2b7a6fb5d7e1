#!/bin/bash
# GEMM epilogue store policy at the step level: JMT_GEMM_DBG=4 (plain stores) vs nontemporal
set -u
OUT=gpurun_out; mkdir -p $OUT
for m in 0 4 0 4; do
  JMT_GEMM_DBG=$m timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-parity --probe-steps 1 > $OUT/store_bench_$m.log 2>&1 || exit 1
  echo "dbg=$m $(grep -o '"ms_per_step": [0-9.]*' $OUT/store_bench_$m.log | head -1)"
done
grep -o '"family": "[a-z_A-Z]*", "launches_per_step": [0-9.]*, "ms_per_step": [0-9.]*, "avg_launch_us": [0-9.]*' $OUT/store_bench_0.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_s3b -o run -- python3 bench.py > $OUT/bench_prof_s3b.log 2>&1
rc=$?; echo "profiled bench exit $rc"; grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' $OUT/bench_prof_s3b.log | head -3
exit $rc
