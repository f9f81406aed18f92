#!/bin/bash
# batched weight-tile / coefficient loads in the fused 1x1 + spatial 3x3 kernels: tests, bench, step timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py tests/test_conv1x1_ks.py tests/test_conv_igemm.py tests/test_bottleneck_block.py -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -15 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
bash tools/gpu_r06e.sh r06o_tl
