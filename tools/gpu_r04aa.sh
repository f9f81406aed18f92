#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 300 python tools/conv1x1_lt_bench.py > $O/conv1x1_lt.jsonl 2>&1 || { tail -5 $O/conv1x1_lt.jsonl; exit 1; }
grep '"m"' $O/conv1x1_lt.jsonl
PMC_FILTER="" bash tools/gpu_pmc_cmd.sh membound tools/pmc_membound.py > gpurun_out/pmc_membound.log 2>&1 || exit 1
tail -1 gpurun_out/pmc_membound.log
