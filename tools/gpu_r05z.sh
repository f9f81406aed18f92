#!/bin/bash
# bn1 dx as conv1's dgrad prologue (recomputed ReLU mask): tests, same-box A/B, bench + trace;
# then which torch copies remain in the step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_bottleneck_block.py tests/test_groupbn.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/ab_bench.sh r05z_bn1pro "APEX_AMD_BN1_DX_PRO=1" "APEX_AMD_BN1_DX_PRO=0" 2 || exit 1
bash tools/gpu_r05b.sh r05z || exit 1
timeout -k 10 300 python -u tools/find_copies.py > $O/copies.txt 2>&1 || { tail -20 $O/copies.txt; exit 1; }
grep -v "^\[bench\]" $O/copies.txt | head -30
