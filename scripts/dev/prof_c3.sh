cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python bench.py --steps 20 --warmup 3 --no-parity --no-cpu-baseline --no-probe > gpurun_out/b_c3_prof.log 2>&1
