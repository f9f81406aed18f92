#!/bin/bash
# column tile fitted to the LDS, channels_last global pool: tests, bench + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_conv1x1_bn.py \
  tests/test_bottleneck_block.py tests/test_standalone_models.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench1.log 2>&1 || exit 1; tail -1 $O/bench1.log | cut -c1-200
bash tools/gpu_r05b.sh r05aa || exit 1
