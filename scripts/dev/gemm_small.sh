# GEMM launches at realdata's row count (1024 tokens per stream): throughput and per-block timeline
set -e
timeout -k 10 120 python scripts/bench_gemm_step.py --rows 1024 --cfg 0 > gpurun_out/gemm_small.jsonl 2>&1
timeout -k 10 120 python scripts/gemm_timeline.py --rows 1024 --only "enc b3 fwd NT" --cfg 0 > gpurun_out/gemm_small_tl.txt 2>&1
timeout -k 10 120 python scripts/gemm_timeline.py --rows 1024 --only "wgrad b3 TN 512" --cfg 0 >> gpurun_out/gemm_small_tl.txt 2>&1
