#!/bin/bash
# MTA unroll A/B (FusedAdam GB/s), optimizer + multi-tensor gpu tests
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
for u in 1 2 1 2; do
  APEX_MTA_UNROLL=$u timeout -k 10 120 python -u tools/bench_kernels.py --only adam > gpurun_out/adam_u$u.jsonl 2>&1
  rc=$?; echo "unroll=$u $(grep fused_adam gpurun_out/adam_u$u.jsonl | cut -c1-160)"; [ $rc -ne 0 ] && stop adam $rc
done
timeout -k 10 300 python -u -m pytest tests/test_optimizers.py tests/test_multi_tensor.py tests/test_amp.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mta.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_mta.log; [ $rc -ne 0 ] && stop pytest $rc
echo ALL_DONE
