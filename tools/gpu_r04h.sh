#!/bin/bash
# native stem: kernel tests vs float64, node bench vs module path, ResNet bench A/B; then the
# transformer benches (GPT-2 medium / BGRADB A/B / BERT-large) and a GPT-2 kernel-trace profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_stem.py > $O/stem_tests.log 2>&1
rc=$?; tail -3 $O/stem_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
if [ $rc -eq 0 ]; then
  timeout -k 10 200 python tools/stem_node_bench.py > $O/stem_bench.log 2>&1 || { tail -5 $O/stem_bench.log; exit 1; }
  cat $O/stem_bench.log
  timeout -k 10 400 python bench.py > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
  tail -1 $O/resnet.log
fi
APEX_AMD_NATIVE_STEM=0 timeout -k 10 400 python bench.py > $O/resnet_nostem.log 2>&1 || { tail -5 $O/resnet_nostem.log; exit 1; }
tail -1 $O/resnet_nostem.log
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_fused_dense.py tests/test_dropout_rng.py tests/test_attention.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2.log 2>&1 || { tail -5 $O/gpt2.log; exit 1; }
tail -1 $O/gpt2.log
APEX_AMD_LT_BGRADB=1 timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2_bgradb.log 2>&1 || { tail -5 $O/gpt2_bgradb.log; exit 1; }
tail -1 $O/gpt2_bgradb.log
timeout -k 10 400 python bench.py --model bert-large --steps 10 --warmup 4 > $O/bert.log 2>&1 || { tail -5 $O/bert.log; exit 1; }
tail -1 $O/bert.log
