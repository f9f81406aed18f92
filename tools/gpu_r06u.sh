#!/bin/bash
# NC=256 column tile (spilling RED epilogue) vs NC=128 at k <= 128: micro-bench + same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 200 python tools/dgrad_bnred_bench.py > $O/dg_a.jsonl 2>&1 || exit 1
APEX_AMD_C1BN_NC256_MAXK=0 timeout -k 10 200 python tools/dgrad_bnred_bench.py > $O/dg_b.jsonl 2>&1 || exit 1
grep '^{' $O/dg_a.jsonl; grep '^{' $O/dg_b.jsonl
bash tools/ab_multi.sh r06u_ab 2 "-" "APEX_AMD_C1BN_NC256_MAXK=0"
