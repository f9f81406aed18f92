#!/bin/bash
# transformer benches on the round-5 tree (GPT-2 medium + FusedAdam, BERT-large + FusedLAMB)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_medium.log 2>&1 || { tail -5 $O/gpt2_medium.log; exit 1; }
tail -1 $O/gpt2_medium.log | cut -c1-220
timeout -k 10 400 python bench.py --model bert-large > $O/bert_large.log 2>&1 || { tail -5 $O/bert_large.log; exit 1; }
tail -1 $O/bert_large.log | cut -c1-220
