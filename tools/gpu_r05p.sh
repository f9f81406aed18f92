#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_bottleneck_block.py > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05p_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05p_nc128 "APEX_AMD_C1BN_NC128_MAXK=512" "APEX_AMD_C1BN_NC128_MAXK=256" 2
