#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters: one rocprofv3 pass per counter group
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), kernel-trace only, then a per-kernel summary.
set -u
TAG=${1:-r02}
OUT=gpurun_out/pmcb_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-parity > $OUT/p$i.log 2>&1 \
      || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summarize.py $OUT gpurun_out/pmc_families_$TAG > $OUT/summary.txt && cat $OUT/summary.txt | head -30
