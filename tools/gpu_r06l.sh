#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l
mkdir -p $O
APEX_AMD_HWG_NW=8 timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_conv_halo_wgrad.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_multi.sh r06l 2 "-" "APEX_AMD_HWG_NW=8"
