set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
timeout -k 10 200 python bench.py --config c3sa --steps 50 --warmup 5 --no-parity > gpurun_out/b_c3sa.log 2>&1
timeout -k 10 200 python bench.py --config realdata --steps 50 --warmup 5 --no-parity > gpurun_out/b_real.log 2>&1
