#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05l
mkdir -p $O
bash tools/gpu_r05b.sh r05l || exit 1
APEX_AMD_BN_CENSUS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 > $O/census.log 2>&1; grep "bn census" $O/census.log | head -40
