set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "forced or gemm" > gpurun_out/t_gemm.log 2>&1
timeout -k 10 300 python scripts/bench_gemm_step.py --rows 1024 --cfg 0 1 26 --reps 30 > gpurun_out/gemm_small26.jsonl 2>&1
timeout -k 10 200 python bench.py --config realdata --steps 50 --warmup 5 --no-parity > gpurun_out/b_real.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1
