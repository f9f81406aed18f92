#!/bin/bash
# BN elementwise passes with per-lane coefficient registers + deeper fused-1x1 ring at k 512:
# tests, BN census, ring-depth A/B, then the driver-exact bench + node trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_groupbn.py \
  tests/test_conv1x1_bn.py tests/test_bottleneck_block.py tests/test_stem.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
APEX_AMD_BN_CENSUS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 > $O/census.log 2>&1; grep "bn census" $O/census.log > $O/census.txt
bash tools/ab_bench.sh r05w_depth "APEX_AMD_C1BN_DEPTH1=4" "APEX_AMD_C1BN_DEPTH1=3" 2 || exit 1
bash tools/gpu_r05b.sh r05w
