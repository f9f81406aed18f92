#!/bin/bash
# KS 1x1 column-tile sweep + the KS GPU tests
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv1x1_ks.py > $O/t_ks.log 2>&1; echo "tests rc=$?"; tail -3 $O/t_ks.log
for nc in auto 64 128 256; do
  if [ $nc = auto ]; then E=""; else E="APEX_AMD_C1KS_NC=$nc"; fi
  env $E timeout -k 10 180 python -u tools/ks_bench.py >> $O/ks_bench.jsonl 2>> $O/ks_bench.err || { echo "bench nc=$nc rc=$?"; exit 1; }
done
cat $O/ks_bench.jsonl
