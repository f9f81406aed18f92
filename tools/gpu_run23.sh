#!/bin/bash
# BN pass tuning: knob sweep on the microbench, groupbn tests, ResNet-50 bench
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
for cfg in "2 4" "4 4" "2 8" "4 8" "8 8"; do
  set -- $cfg
  APEX_BN_BLOCKS_PER_CU=$1 APEX_BN_BWD_ROWS=$2 timeout -k 10 120 python -u tools/bn_bench.py >> gpurun_out/bn_bench.jsonl 2>&1
  rc=$?; [ $rc -ne 0 ] && stop bn_bench $rc
done
grep total gpurun_out/bn_bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_groupbn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bn.log; [ $rc -ne 0 ] && stop pytest $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -ne 0 ] && stop bench $rc
echo ALL_DONE
