#!/bin/bash
# MHA fast path on the packed-QKV kernels: attention GPU tests, the published-config perf test
# (host enqueue cost + hipGraph replay rows); GPT-2 medium A/B of the hipBLASLt plan tuning
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_attention.py > $O/attn_tests.log 2>&1
rc=$?; tail -2 $O/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/perf_test_multihead_attn.py --graph --out $O/mha_published_config.jsonl > $O/mha.log 2>&1 || { tail -5 $O/mha.log; exit 1; }
cat $O/mha.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2_tune_$i.log 2>&1 || { tail -5 $O/gpt2_tune_$i.log; exit 1; }
  tail -1 $O/gpt2_tune_$i.log | cut -c1-200
  APEX_AMD_LT_TUNE=0 timeout -k 10 400 python bench.py --model gpt2-medium --steps 10 --warmup 4 > $O/gpt2_notune_$i.log 2>&1 || { tail -5 $O/gpt2_notune_$i.log; exit 1; }
  tail -1 $O/gpt2_notune_$i.log | cut -c1-200
done
