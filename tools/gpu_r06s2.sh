#!/bin/bash
# round 6: stride-2 halo weight gradient — GPU tests, micro-bench vs MIOpen, same-box step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06s2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_halo_wgrad.py -m gpu \
  > $O/test_hwg.txt 2>&1 || { tail -30 $O/test_hwg.txt; exit 1; }
tail -2 $O/test_hwg.txt
timeout -k 10 200 python tools/wgrad_s2_bench.py > $O/wgrad_s2.jsonl 2>&1 || { tail -20 $O/wgrad_s2.jsonl; exit 1; }
cat $O/wgrad_s2.jsonl
tools/ab_bench.sh r06s2/ab3 "APEX_AB_NOP=1" "APEX_AMD_HALO_WGRAD_S2=0" 2
