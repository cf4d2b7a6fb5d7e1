#!/bin/bash
# Round-3 evidence of one build: smoke, the plain default bench, the same command under
# rocprofv3 (kernel trace + stats) -> per-family timed-region trace JSON, then the PMC HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE separately).  JMT_COMMIT stamps the JSON files.
set -u
TAG=${1:-p1}
OUT=gpurun_out/r03/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --launch-log $OUT/launch_log.jsonl > $OUT/bench_plain.log 2>&1 || { echo bench failed; tail $OUT/bench_plain.log; exit 1; }
grep '^{' $OUT/bench_plain.log | tail -1 | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { echo prof failed; tail $OUT/bench_prof.log; exit 1; }
db=$(find $OUT/prof -name "*results.db" | head -1)
python scripts/family_from_trace.py "$db" $OUT/bench_prof.log --json $OUT/family_trace.json > $OUT/family_check.txt 2>&1
cat $OUT/family_check.txt
find $OUT/prof -name "*.db" -delete
find $OUT/prof -name "*kernel_trace.csv" -delete
mkdir -p $OUT/pmc
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $OUT/pmc/p$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-probe --no-parity > $OUT/pmc/p$i.log 2>&1 \
      || { echo "pmc pass $i failed"; tail -5 $OUT/pmc/p$i.log; exit 1; }
done
python3 scripts/pmc_summarize.py $OUT/pmc $OUT/pmc_families > $OUT/pmc_summary.txt && head -8 $OUT/pmc_summary.txt | cut -c1-200
find $OUT/pmc -name "*.csv" -size +2M -delete
