#!/bin/bash
# A/B sweep of the NHWC batch-norm partial-pass occupancy (tools/bn_bench.py per setting)
mkdir -p gpurun_out
for cfg in "2 2" "4 2" "8 2" "4 4" "8 4"; do
  set -- $cfg
  APEX_BN_STATS_BPC=$1 APEX_BN_BWD_BPC=$2 timeout -k 10 120 python tools/bn_bench.py > gpurun_out/bn_sweep_$1_$2.log 2>&1 || exit $?
  echo "stats_bpc=$1 bwd_bpc=$2: $(tail -1 gpurun_out/bn_sweep_$1_$2.log)"
done
