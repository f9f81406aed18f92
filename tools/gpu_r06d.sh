#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_conv1x1_ks.py \
  > $O/tests_ks.log 2>&1
rc=$?; tail -3 $O/tests_ks.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_bottleneck_block.py \
  tests/test_standalone_models.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_multi.sh r06g 2 "-" "APEX_AMD_C1KS=0" "APEX_AMD_C1KS_PRO=1"
