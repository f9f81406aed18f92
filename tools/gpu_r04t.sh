#!/bin/bash
# Deferred block output (ResNet) + pair-hash attention dropout + hipBLASLt mm routes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
  tests/test_bottleneck_block.py tests/test_conv1x1_bn.py tests/test_conv3_bwd.py tests/test_stem.py tests/test_attention.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/attn_dropout_bench.py > $O/attn_dropout.jsonl 2>&1 || { tail -5 $O/attn_dropout.jsonl; exit 1; }
cut -c1-200 $O/attn_dropout.jsonl
timeout -k 10 400 python bench.py > $O/resnet_defer.log 2>&1 || { tail -5 $O/resnet_defer.log; exit 1; }
tail -1 $O/resnet_defer.log | cut -c1-160
APEX_AMD_DEFER_OUTPUT=0 timeout -k 10 400 python bench.py > $O/resnet_nodefer.log 2>&1 || { tail -5 $O/resnet_nodefer.log; exit 1; }
tail -1 $O/resnet_nodefer.log | cut -c1-160
timeout -k 10 300 python tools/gemm_route_bench.py > $O/gemm_routes.jsonl 2>&1 || { tail -5 $O/gemm_routes.jsonl; exit 1; }
cut -c1-400 $O/gemm_routes.jsonl
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2.log 2>&1 || { tail -5 $O/gpt2.log; exit 1; }
tail -1 $O/gpt2.log | cut -c1-160
