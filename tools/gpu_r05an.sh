#!/bin/bash
# same-box A/B: multi-tensor work-item size in the ResNet-50 step (FusedAdam over 25.6M params)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_bench.sh r05an_item "APEX_AMD_MTA_ITEM=8192" "APEX_AMD_MTA_ITEM=16384" 2 || exit 1
