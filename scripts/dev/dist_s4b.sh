#!/bin/bash
# localise the slow 2-rank gloo rehearsal: overlap off / side stream off / both
set -u
OUT=gpurun_out/dist; mkdir -p $OUT
run() {  # tag, env, args
  env $2 JMT_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $4 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --probe-steps 1 $3 > $OUT/d_$1.log 2>&1
  rc=$?; echo "$1 exit $rc $(grep -o '"ms_per_step": [0-9.]*\|"host_issue_ms_per_eager_step": [0-9.]*' $OUT/d_$1.log | tr '\n' ' ')"
  return $rc
}
run base "JMT_X=1" "" 29531 && run nooverlap "JMT_X=1" "--no-overlap" 29532 && run noside "JMT_SIDE_STREAM=0" "" 29533 && run noside_nooverlap "JMT_SIDE_STREAM=0" "--no-overlap" 29534
