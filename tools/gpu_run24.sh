#!/bin/bash
mkdir -p gpurun_out
stop() { echo "STOP: $1 rc=$2"; exit $2; }
for f in 0 1 0 1; do
  APEX_BN_EW_FIXED=$f timeout -k 10 120 python -u tools/bn_bench.py > gpurun_out/bn_ab_$f.jsonl 2>&1
  rc=$?; [ $rc -ne 0 ] && stop bn_bench $rc
  echo "fixed=$f $(grep total gpurun_out/bn_ab_$f.jsonl)"
done
echo ALL_DONE
