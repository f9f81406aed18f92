#!/bin/bash
# Deferred block-output fusion: bottleneck / 1x1 / stem / conv3 tests, ResNet bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
  tests/test_bottleneck_block.py tests/test_conv1x1_bn.py tests/test_conv3_bwd.py tests/test_stem.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python bench.py > $O/resnet_defer.log 2>&1 || { tail -5 $O/resnet_defer.log; exit 1; }
tail -1 $O/resnet_defer.log | cut -c1-200
APEX_AMD_DEFER_OUTPUT=0 timeout -k 10 400 python bench.py > $O/resnet_nodefer.log 2>&1 || { tail -5 $O/resnet_nodefer.log; exit 1; }
tail -1 $O/resnet_nodefer.log | cut -c1-200
timeout -k 10 300 python tools/gemm_route_bench.py > $O/gemm_routes.jsonl 2>&1 || { tail -5 $O/gemm_routes.jsonl; exit 1; }
cut -c1-400 $O/gemm_routes.jsonl
