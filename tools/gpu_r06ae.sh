#!/bin/bash
# fused 1x1 operand-ring depth now that the rings are scratch-free: same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_multi.sh r06ae_ab 2 "-" "APEX_AMD_C1BN_DEPTH1=5" "APEX_AMD_C1BN_DEPTH1=3" "APEX_AMD_C1BN_DEPTH=3" || exit 1
