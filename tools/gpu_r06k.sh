#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_conv_igemm.py \
  tests/test_bottleneck_block.py tests/test_conv1x1_bn.py tests/test_conv1x1_ks.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_multi.sh r06k 2 "-" "APEX_AMD_BN1_RED=0"
