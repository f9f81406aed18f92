#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_bottleneck_block.py \
  tests/test_conv1x1_bn.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_multi.sh r06c 2 "-" "APEX_AMD_DS_DX_PRO=0 APEX_AMD_DS_RED=0" "APEX_AMD_CONV_HFP=0"
