#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python -u tools/bn1_fold_bench.py > $O/fold.jsonl 2>&1; grep shape $O/fold.jsonl
bash tools/ab_bench.sh r05o_nc "APEX_AMD_C1BN_NC256_MAXK=256" "APEX_AMD_C1BN_NC256_MAXK=128" 2
