#!/bin/bash
# channel-padded stem: tests, bench x2
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_conv1x1.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_conv.log; [ $rc -ne 0 ] && stop pytest $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_stem$i.log 2>&1
  rc=$?; echo "$(tail -1 gpurun_out/bench_stem$i.log | cut -c1-120)"; [ $rc -ne 0 ] && stop bench $rc
done
echo ALL_DONE
