#!/bin/bash
# native 1x1 conv routing: tests, A/B bench; then MIOpen full-find experiment
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_conv1x1.py tests/test_standalone_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_conv.log; [ $rc -ne 0 ] && stop pytest $rc
for f in 0 1 0 1; do
  APEX_AMD_CONV1X1=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_conv$f.log 2>&1
  rc=$?; echo "conv1x1=$f $(tail -1 gpurun_out/bench_conv$f.log | cut -c1-120)"; [ $rc -ne 0 ] && stop bench $rc
done
s=$(date +%s)
MIOPEN_FIND_MODE=NORMAL timeout -k 10 600 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_findnormal.log 2>&1
rc=$?; e=$(date +%s); echo "findnormal wall=$((e-s))s $(tail -1 gpurun_out/bench_findnormal.log | cut -c1-120)"; [ $rc -ne 0 ] && stop find $rc
echo ALL_DONE
