set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/b_c3.log 2>&1
timeout -k 10 200 python bench.py --config c3sa --steps 50 --warmup 5 --no-parity > gpurun_out/b_c3sa.log 2>&1
JMT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 --config realdata --scaling strong > gpurun_out/b_dist2s.log 2>&1
