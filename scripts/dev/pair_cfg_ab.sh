# MLP pair A/B on the c5 (digitized k=20, fp16, B=128) and c4 (T=1024) workloads, interleaved
set -e
mkdir -p gpurun_out/pcfg
for c in c5 c4; do
  for m in 0 1 0 1; do
    JMT_PAIR_MLP=$m timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-parity --probe-steps 1 > gpurun_out/pcfg/${c}_$m.log 2>&1
    echo "$c pair=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pcfg/${c}_$m.log | head -1)"
  done
done
