#!/bin/bash
# Interleaved step A/B on one box: bench.py (c3 unless CONFIG is set) under each environment in
# turn, ROUNDS rounds, ms/step per run.  Usage: scripts/ab_step.sh OUT "ENV_A" "ENV_B" ...
# (an environment is a space-separated list of VAR=value, or "-" for the defaults)
OUT=$1; shift
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    envs=(); [ "$e" != "-" ] && envs=($e)
    ms=$(env "${envs[@]}" timeout -k 10 150 python -u bench.py --config ${CONFIG:-c3} --steps ${STEPS:-100} \
         --warmup 5 --no-probe --no-parity --no-cpu-baseline 2>/dev/null | tail -1 |
         python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "round $r  env [$e]  ${CONFIG:-c3}  $ms ms/step" | tee -a "$OUT"
  done
done
