#!/bin/bash
# bn1 apply + ReLU folded into the halo-staged 3x3 kernels (spatial fprop, halo fprop, halo wgrad):
# bitwise prologue tests, block / chain tests, headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_halo_wgrad.py \
  tests/test_conv_halo_fprop.py tests/test_bottleneck_block.py tests/test_groupbn.py tests/test_syncbn.py > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05n_fold "APEX_AMD_BN1_FOLD=0" "APEX_AMD_BN1_FOLD=1" 2
