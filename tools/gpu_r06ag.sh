#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_multi.sh r06ag_ab 2 "-" "APEX_AMD_BN1_DX_PRO=1" "APEX_AMD_BN1_FOLD=1" "APEX_AMD_BN1_RED=1" "APEX_AMD_C1KS=1" || exit 1
