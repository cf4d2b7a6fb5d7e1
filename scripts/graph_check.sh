#!/bin/bash
# hipGraph whole-step capture: parity test + bench graph vs eager (+ streams inside the capture)
set -u
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-g}
JMT_CAPTURE_STREAMS=${JMT_CAPTURE_STREAMS:-1} timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_graph_tests.log 2>&1
rc=$?; echo "graph tests exit $rc"; tail -6 $OUT/${TAG}_graph_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for mode in "--graph" "--no-graph"; do
  JMT_CAPTURE_STREAMS=${JMT_CAPTURE_STREAMS:-1} timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $mode > $OUT/${TAG}_bench${mode}.log 2>&1
  rc=$?; echo "bench $mode exit $rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"host_issue_ms_per_eager_step": [0-9.]*\|"frac": [0-9.]*' $OUT/${TAG}_bench${mode}.log | tr '\n' ' '; echo
  if [ $rc -ne 0 ]; then tail -20 $OUT/${TAG}_bench${mode}.log; exit $rc; fi
done
JMT_CAPTURE_STREAMS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_bench_nostreams.log 2>&1
rc=$?; echo "bench graph, no capture streams exit $rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $OUT/${TAG}_bench_nostreams.log | tr '\n' ' '; echo
exit $rc
