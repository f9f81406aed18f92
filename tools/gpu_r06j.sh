#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_multi.sh r06j 2 "APEX_AMD_BN1_RED=0" "APEX_AMD_BN1_RED=0 APEX_AMD_S2_DGRAD_128=1"
