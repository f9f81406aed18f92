#!/bin/bash
# attention forward occupancy / query-fragment variants (the default spills 46 VGPRs with the
# bias + dropout mode at d = 64): same-box A/B on BERT-large and GPT-2 medium
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--model bert-large" bash tools/ab_multi.sh r06x_bert 2 "-" "APEX_ATTN_FWD_OCC=lo" "APEX_ATTN_FWD_QF=2" || exit 1
BENCH_ARGS="--model gpt2-medium" bash tools/ab_multi.sh r06x_gpt2 2 "-" "APEX_ATTN_FWD_OCC=lo" "APEX_ATTN_FWD_QF=2" || exit 1
