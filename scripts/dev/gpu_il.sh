#!/bin/bash
# GPU check of the interleaved-issue GEMM configs (6, 7) and the interleaved attention staging:
# forced-config GEMM numerics, model parity, per-block timeline, shape sweep, attention, bench.
set -u
O=gpurun_out; mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
JMT_GEMM_CFG=6 timeout -k 10 300 $T tests/test_gpu_kernels.py -k gemm > $O/il_t6.log 2>&1 || { echo "cfg6 tests failed"; tail -30 $O/il_t6.log; exit 1; }
JMT_GEMM_CFG=7 timeout -k 10 300 $T tests/test_gpu_kernels.py -k gemm > $O/il_t7.log 2>&1 || { echo "cfg7 tests failed"; tail -30 $O/il_t7.log; exit 1; }
timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_graph.py > $O/il_tm.log 2>&1 || { echo "model tests failed"; tail -30 $O/il_tm.log; exit 1; }
tail -2 $O/il_tm.log
timeout -k 10 200 python scripts/gemm_timeline.py --only "fwd NT 512" --cfg 5 6 7 > $O/il_tl.log 2>&1 || exit 1
grep cfg $O/il_tl.log | grep -v shape
timeout -k 10 300 python scripts/bench_gemm_step.py --cfg 5 6 7 > $O/il_gs.log 2>&1 || exit 1
grep shape $O/il_gs.log
timeout -k 10 200 python scripts/bench_attn.py > $O/il_attn.log 2>&1 || exit 1
grep fused $O/il_attn.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/il_bench.log 2>&1 || exit 1
tail -c 600 $O/il_bench.log
