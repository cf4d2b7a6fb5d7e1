set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/b_c3.log 2>&1
