#!/bin/bash
# N>1 bench path rehearsal on the current build: 2 and 4 ranks sharing the one GPU over gloo
# (sharding, global-batch CCC all-gather, overlapped bucketed all-reduce, max-over-ranks timing);
# numbers are not a measurement (ranks share one GPU, gloo stages through the host)
set -u
OUT=gpurun_out/dist; mkdir -p $OUT
for n in 2 4; do
  JMT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline > $OUT/dist$n.log 2>&1
  rc=$?; echo "dist$n exit $rc"; grep '^{' $OUT/dist$n.log | tail -1 | cut -c1-420
  if [ $rc -ne 0 ]; then tail -20 $OUT/dist$n.log; exit $rc; fi
done
JMT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29520 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --scaling strong > $OUT/dist2_strong.log 2>&1
rc=$?; echo "dist2 strong exit $rc"; grep '^{' $OUT/dist2_strong.log | tail -1 | cut -c1-420
exit $rc
