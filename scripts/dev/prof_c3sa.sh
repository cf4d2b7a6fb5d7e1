cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3sa -o run -- python bench.py --config c3sa --steps 20 --warmup 3 --no-parity --no-cpu-baseline --no-probe > gpurun_out/b_c3sa_prof.log 2>&1
