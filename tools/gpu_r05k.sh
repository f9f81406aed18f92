#!/bin/bash
# A/B of the halo-tile 3x3 fprop at 7x7 (APEX_AMD_CONV_HFP=0: the tap GEMM everywhere) on the
# native-everywhere 1x1 default
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_bench.sh r05k_hfp "APEX_AMD_CONV_HFP=1" "APEX_AMD_CONV_HFP=0" 2
