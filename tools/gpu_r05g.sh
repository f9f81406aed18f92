#!/bin/bash
# strided 1x1 downsample through the stride-2 subsample + native 1x1 kernels: kernel + block tests,
# then the headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_bottleneck_block.py > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05g_ds "APEX_AMD_DS_SUBSAMPLE=0" "APEX_AMD_DS_SUBSAMPLE=1" 2
