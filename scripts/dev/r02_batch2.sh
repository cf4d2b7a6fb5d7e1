set -e
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py "tests/test_gpu_models.py::test_attention_class_callable" "tests/test_gpu_configs.py::test_c5_expression_head_fp16_vs_oracle" > gpurun_out/t_dist.log 2>&1
python -c "import json,sys; sys.path[:0]=['.','joint-multimodal-transformer-6th-abaw_amd']; from tests.test_config import _schema; json.dump(_schema(), open('/tmp/cfg.json','w'))"
timeout -k 10 200 python bench.py --config-file /tmp/cfg.json --num_heads 2 --steps 30 --warmup 3 > gpurun_out/b_cfgfile.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 30 --warmup 3 > gpurun_out/b_c5.log 2>&1
