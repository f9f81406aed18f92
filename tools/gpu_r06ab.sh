#!/bin/bash
# tap-image prefetch + 256-column tiles at k <= 64 (non-RED): tests, same-box A/B, timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ab; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_bottleneck_block.py tests/test_conv_igemm.py tests/test_bottleneck.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_multi.sh r06ab_ab 2 "-" "APEX_AMD_TAP_PREFETCH=0" "APEX_AMD_C1BN_NC256_MAXK=0" || exit 1
bash tools/gpu_r06e.sh r06ab_tl > /dev/null || exit 1
