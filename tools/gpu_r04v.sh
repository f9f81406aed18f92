#!/bin/bash
# fused1x1 prefetch ring depth 2 vs 3: tests, per-shape kernel times, ResNet A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
  tests/test_conv1x1_bn.py tests/test_bottleneck_block.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
APEX_AMD_C1BN_DEPTH=2 timeout -k 10 300 python tools/bn1x1_bench.py --rounds 2 > $O/bn1x1_d2.jsonl 2>&1 || { tail -5 $O/bn1x1_d2.jsonl; exit 1; }
APEX_AMD_C1BN_DEPTH=3 timeout -k 10 300 python tools/bn1x1_bench.py --rounds 2 > $O/bn1x1_d3.jsonl 2>&1 || { tail -5 $O/bn1x1_d3.jsonl; exit 1; }
timeout -k 10 400 python bench.py > $O/resnet_d3.log 2>&1 || { tail -5 $O/resnet_d3.log; exit 1; }
tail -1 $O/resnet_d3.log | cut -c1-160
APEX_AMD_C1BN_DEPTH=2 timeout -k 10 400 python bench.py > $O/resnet_d2.log 2>&1 || { tail -5 $O/resnet_d2.log; exit 1; }
tail -1 $O/resnet_d2.log | cut -c1-160
timeout -k 10 400 python bench.py > $O/resnet_d3b.log 2>&1 || { tail -5 $O/resnet_d3b.log; exit 1; }
tail -1 $O/resnet_d3b.log | cut -c1-160
