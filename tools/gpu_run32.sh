#!/bin/bash
# ReLU bit mask for residual add+ReLU BN: tests, pass microbench A/B, ResNet-50 A/B
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_groupbn.py tests/test_standalone_models.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bn.log; [ $rc -ne 0 ] && stop pytest $rc
for f in 0 1; do
  APEX_BN_BITS=$f timeout -k 10 120 python -u tools/bn_bench.py > gpurun_out/bn_bits$f.jsonl 2>&1
  rc=$?; echo "bits=$f $(grep total gpurun_out/bn_bits$f.jsonl)"; [ $rc -ne 0 ] && stop bn_bench $rc
done
for f in 0 1 0 1; do
  APEX_BN_BITS=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 > gpurun_out/bench_bits$f.log 2>&1
  rc=$?; echo "bits=$f $(tail -1 gpurun_out/bench_bits$f.log | cut -c60-120)"; [ $rc -ne 0 ] && stop bench $rc
done
echo ALL_DONE
