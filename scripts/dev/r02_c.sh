set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "small or attention_core" tests/test_gpu_models.py tests/test_gpu_configs.py > gpurun_out/t_c.log 2>&1
timeout -k 10 200 python bench.py --config c3sa --steps 50 --warmup 5 --no-parity > gpurun_out/b_c3sa.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-parity --no-cpu-baseline > gpurun_out/b_c3.log 2>&1
