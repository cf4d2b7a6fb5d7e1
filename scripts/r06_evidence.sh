#!/bin/bash
# Round-6 evidence at the benched commit (JMT_COMMIT=<hash>; the GPU box has no .git):
#  1. rocprofv3 --kernel-trace --stats over the default bench command (200 timed steps) ->
#     kernel_stats.csv, the per-family in-step trace (scripts/family_from_trace.py --json)
#  2. per-family HBM traffic from FETCH_SIZE / WRITE_SIZE in separate PMC passes
#     (scripts/pmc_bench.sh -> traffic_<family>.json, gfx950 FETCH_SIZE x2 correction)
set -u
C=${JMT_COMMIT:?set JMT_COMMIT}
OUT=gpurun_out/r06/ev_$C
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline > $OUT/bench_under_rocprof.log 2>&1 \
    || { echo "rocprof bench failed"; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
db=$(find $OUT/prof -name "*results.db" | head -1)
stats=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
echo "db $db stats $stats"
cp "$stats" $OUT/kernel_stats.csv
python3 scripts/family_from_trace.py "$db" $OUT/bench_under_rocprof.log \
    --json $OUT/family_trace.json > $OUT/family_trace.txt 2>&1 || { cat $OUT/family_trace.txt; exit 1; }
cat $OUT/family_trace.txt
bash scripts/pmc_bench.sh r06_$C || exit 1
cp -r gpurun_out/pmc_families_r06_$C $OUT/pmc_families
cp gpurun_out/pmcb_r06_$C/summary.txt $OUT/pmc_summary.txt
rm -rf $OUT/prof gpurun_out/pmcb_r06_$C/p1 gpurun_out/pmcb_r06_$C/p2
