set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu_all.log 2>&1
python -c "import json,sys; sys.path[:0]=['.','joint-multimodal-transformer-6th-abaw_amd']; from tests.test_config import _schema; json.dump(_schema(), open('/tmp/cfg.json','w'))"
timeout -k 10 200 python bench.py --config-file /tmp/cfg.json --num_heads 2 --steps 30 --warmup 3 > gpurun_out/b_cfgfile.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 30 --warmup 3 > gpurun_out/b_c5.log 2>&1
