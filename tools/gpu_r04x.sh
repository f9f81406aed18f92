#!/bin/bash
# spatial-tile 3x3 kernel: its own tests first (new kernel), conv tests, microbench, ResNet A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04x3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread \
  tests/test_conv_igemm.py -k spatial > $O/tests_sp.log 2>&1 || { tail -30 $O/tests_sp.log; exit 1; }
tail -2 $O/tests_sp.log
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
  tests/test_conv_igemm.py tests/test_conv1x1_bn.py tests/test_bottleneck_block.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/conv_sp_bench.py > $O/conv_sp.jsonl 2>&1 || { tail -5 $O/conv_sp.jsonl; exit 1; }
cat $O/conv_sp.jsonl | grep arm
timeout -k 10 400 python bench.py > $O/resnet_sp.log 2>&1 || { tail -5 $O/resnet_sp.log; exit 1; }
tail -1 $O/resnet_sp.log | cut -c1-160
APEX_AMD_CONV_SP=0 timeout -k 10 400 python bench.py > $O/resnet_nosp.log 2>&1 || { tail -5 $O/resnet_nosp.log; exit 1; }
tail -1 $O/resnet_nosp.log | cut -c1-160
