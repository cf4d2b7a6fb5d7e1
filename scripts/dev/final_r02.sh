# final round-2 evidence: PMC traffic passes, then the default bench command under rocprofv3
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/pmc_bench.sh r02 > gpurun_out/pmc.log 2>&1
mkdir -p profiles/r02_pmc_bench && cp gpurun_out/pmc_families_r02/*.json profiles/r02_pmc_bench/
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python bench.py > gpurun_out/bench_prof.log 2>&1
