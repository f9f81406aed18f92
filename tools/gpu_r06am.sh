#!/bin/bash
# knob sweep on the final tree (same box, 2 rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_multi.sh r06am_ab 2 "-" "APEX_AMD_C1BN_NC128_MAXK=256" "APEX_AMD_WGRAD_RING=1" "APEX_AMD_HWG_NW=4" "APEX_AMD_CONV_HFP=1" || exit 1
