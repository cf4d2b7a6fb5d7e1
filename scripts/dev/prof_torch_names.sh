cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_torch -o run -- python scripts/dev/torch_gemm_names.py > gpurun_out/torch_names.log 2>&1
