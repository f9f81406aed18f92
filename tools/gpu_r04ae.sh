#!/bin/bash
# GPT-2 medium: tensor-parallel linear forward route A/B (lt timed plans / torch addmm / native)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ae
mkdir -p $O
for r in lt torch native; do
  APEX_AMD_TP_LINEAR=$r timeout -k 10 400 python bench.py --model gpt2-medium > $O/gpt2_$r.log 2>&1 || { tail -5 $O/gpt2_$r.log; exit 1; }
  echo "$r $(tail -1 $O/gpt2_$r.log | cut -c1-120)"
done
