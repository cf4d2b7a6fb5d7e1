#!/bin/bash
set -u
for c in torch_fork torch_fork_record torch_autograd jmt_linear jmt_linear_bwd; do
  timeout -k 5 120 python scripts/dev/capture_probe.py $c > gpurun_out/cap_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; tail -2 gpurun_out/cap_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
