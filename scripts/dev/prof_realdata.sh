cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 150 python bench.py --config realdata --steps 50 --warmup 5 --no-parity --launch-log gpurun_out/real_launches.jsonl > gpurun_out/b_real.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_real -o run -- python bench.py --config realdata --steps 50 --warmup 5 --no-parity --no-probe > gpurun_out/b_real_prof.log 2>&1
