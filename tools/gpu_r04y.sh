#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 200 python tools/dbg_sp_chain.py > $O/dbg_sp.log 2>&1 || { tail -20 $O/dbg_sp.log; exit 1; }
grep -v amdgpu.ids $O/dbg_sp.log
APEX_AMD_CONV_SP=0 timeout -k 10 200 python tools/dbg_sp_chain.py > $O/dbg_nosp.log 2>&1 || { tail -20 $O/dbg_nosp.log; exit 1; }
grep -v amdgpu.ids $O/dbg_nosp.log
timeout -k 10 200 python tools/conv_sp_bench.py > $O/conv_sp.jsonl 2>&1 || { tail -5 $O/conv_sp.jsonl; exit 1; }
grep arm $O/conv_sp.jsonl
