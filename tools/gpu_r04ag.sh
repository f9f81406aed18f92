#!/bin/bash
# same-box A/B of the fused LayerNorm + residual-gradient node (GPT-2 medium, BERT-large)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x -m gpu --timeout 150 --timeout-method thread tests/test_norm.py tests/test_standalone_models.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1; do
  APEX_AMD_LN_RESIDUAL=$v timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_ln$v.log 2>&1 || { tail -5 $O/gpt2_ln$v.log; exit 1; }
  echo "gpt2 ln_res=$v $(tail -1 $O/gpt2_ln$v.log | cut -c80-130)"
done
for v in 1 0; do
  APEX_AMD_LN_RESIDUAL=$v timeout -k 10 400 python bench.py --model bert-large > $O/bert_ln$v.log 2>&1 || { tail -5 $O/bert_ln$v.log; exit 1; }
  echo "bert ln_res=$v $(tail -1 $O/bert_ln$v.log | cut -c80-130)"
done
