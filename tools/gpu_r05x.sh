#!/bin/bash
# native dgrad weight image (tap_weights), stem pool strip height: tests, A/B, bench + node trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_conv_igemm.py tests/test_stem.py tests/test_bottleneck_block.py tests/test_conv_halo_fprop.py \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05x_pr "APEX_AMD_STEM_PR=4" "APEX_AMD_STEM_PR=2" 2 || exit 1
bash tools/gpu_r05b.sh r05x
