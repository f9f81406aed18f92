#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
APEX_AMD_HWG_NW=8 bash tools/gpu_r06e.sh r06m > /dev/null || exit 1
grep -n "hwg::" gpurun_out/r06m/timeline.md | awk -F'|' '{print $2, $3, $4, $6}' | cut -c1-150
