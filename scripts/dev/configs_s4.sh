# other BASELINE workloads on the final round-2 build (MLP pair): 50 graphed steps each
set -e
mkdir -p gpurun_out/cfg
for c in c2 c4 c5 c3sa realdata; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/cfg/$c.log 2>&1
  grep '^{' gpurun_out/cfg/$c.log | tail -1 >> gpurun_out/cfg/configs_s4.jsonl
  echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*\|"pass": [a-z]*' gpurun_out/cfg/$c.log | tr '\n' ' ')"
done
