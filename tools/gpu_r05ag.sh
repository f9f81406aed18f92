#!/bin/bash
# same-box A/B: one RNG-step snapshot per step vs one per dropout call (GPT-2 medium, BERT-large)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag
mkdir -p $O
for i in 1 2; do
  for arm in 1 0; do
    APEX_AMD_RNG_SHARED_SNAPSHOT=$arm timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_${arm}_$i.log 2>&1 || exit 1
    echo "gpt2 shared=$arm round $i: $(tail -1 $O/gpt2_${arm}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
  done
done
for arm in 1 0; do
  APEX_AMD_RNG_SHARED_SNAPSHOT=$arm timeout -k 10 400 python bench.py --model bert-large > $O/bert_${arm}.log 2>&1 || exit 1
  echo "bert shared=$arm: $(tail -1 $O/bert_${arm}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
done
