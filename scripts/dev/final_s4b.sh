# round-2 final evidence (session 4, MLP-pair build): smoke, the plain default bench command, the
# same command under rocprofv3 (kernel trace + stats) and the per-family trace attribution
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s4b
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4b/smoke.log 2>&1
tail -1 gpurun_out/s4b/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/s4b/bench_plain.log 2>&1
grep '^{' gpurun_out/s4b/bench_plain.log | tail -1 | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s4b/prof -o run -- python3 bench.py > gpurun_out/s4b/bench_prof.log 2>&1
db=$(find gpurun_out/s4b/prof -name "*results.db" | head -1)
python scripts/family_from_trace.py "$db" gpurun_out/s4b/bench_prof.log > gpurun_out/s4b/family_check.txt 2>&1 || true
find gpurun_out/s4b/prof -name "*.db" -delete
find gpurun_out/s4b/prof -name "*kernel_trace.csv" -delete
