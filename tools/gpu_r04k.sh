#!/bin/bash
# producer/consumer conv3 backward: tests, microbench vs the two-kernel path, ResNet bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_conv3_bwd.py tests/test_bottleneck_block.py -k "conv3 or matches_fp32" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/conv3_bwd_bench.py > $O/c3b_bench.log 2>&1 || { tail -5 $O/c3b_bench.log; exit 1; }
cat $O/c3b_bench.log
timeout -k 10 400 python bench.py > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
tail -1 $O/resnet.log | cut -c1-200
