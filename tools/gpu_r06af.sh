#!/bin/bash
# re-A/B of the opt-in node fusions on the scratch-free tree (they were measured while the fused
# 1x1 rings / reduction epilogues still spilled)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_multi.sh r06af_ab 2 "-" "APEX_AMD_BN1_DX_PRO=1" "APEX_AMD_BN1_FOLD=1" "APEX_AMD_BN1_RED=1" "APEX_AMD_C1KS=1" || exit 1
