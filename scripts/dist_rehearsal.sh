#!/bin/bash
# Rehearsal of bench.py's N>1 path (sharding, global-batch CCC all-gather, grad all-reduce,
# max-over-ranks timing) with 2 ranks on a 1-GPU box over gloo; the numbers are not a
# measurement (two ranks share one GPU and gloo stages through the host).
set -u
OUT=gpurun_out; mkdir -p $OUT
JMT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/dist2.log 2>&1
rc=$?; echo "dist2 exit $rc"; tail -1 $OUT/dist2.log | cut -c1-300
exit $rc
