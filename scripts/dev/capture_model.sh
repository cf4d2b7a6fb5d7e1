#!/bin/bash
set -u
for mode in relaxed; do
  CAPMODE=$mode AMD_LOG_LEVEL=1 timeout -k 5 120 python -X faulthandler scripts/dev/capture_model.py fwdbwd > gpurun_out/capm_$mode.log 2>&1
  rc=$?; echo "$mode rc=$rc"; grep -v "^  File\|^Thread\|^$" gpurun_out/capm_$mode.log | head -20
  if [ $rc -ne 0 ]; then exit $rc; fi
done
