set -e
for c in c2 c4 c5 c3sa realdata; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/cfg_$c.log 2>&1
  grep '^{' gpurun_out/cfg_$c.log | tail -1 >> gpurun_out/configs_r02.jsonl
done
