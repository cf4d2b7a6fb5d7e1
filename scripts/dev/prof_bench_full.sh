# the default bench command under rocprofv3 (kernel trace + stats), then the plain command
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python bench.py > gpurun_out/bench_prof.log 2>&1
