# round-2 session-4 evidence on the final build: the plain default bench command, then the same
# command under rocprofv3 (kernel trace + stats) with the per-family trace attribution
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s4
timeout -k 10 400 python bench.py > gpurun_out/s4/bench_plain.log 2>&1
grep '^{' gpurun_out/s4/bench_plain.log | tail -1 | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof -o run -- python3 bench.py > gpurun_out/s4/bench_prof.log 2>&1
db=$(find gpurun_out/s4/prof -name "*results.db" | head -1)
python scripts/family_from_trace.py "$db" gpurun_out/s4/bench_prof.log > gpurun_out/s4/family_check.txt 2>&1 || true
python scripts/kstats.py $(find gpurun_out/s4/prof -name "*kernel_stats.csv" | head -1) > gpurun_out/s4/kstats.txt 2>&1 || cp $(find gpurun_out/s4/prof -name "*kernel_stats.csv" | head -1) gpurun_out/s4/kernel_stats.csv || true
find gpurun_out/s4/prof -name "*.db" -delete
find gpurun_out/s4/prof -name "*kernel_trace.csv" -delete
