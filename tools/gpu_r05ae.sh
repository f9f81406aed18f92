#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05ae
timeout -k 10 400 python -u tools/find_copies.py --model gpt2-medium > gpurun_out/r05ae/copies.txt 2>&1 || { tail -20 gpurun_out/r05ae/copies.txt; exit 1; }
grep "\[agg\]" -A3 gpurun_out/r05ae/copies.txt | head -60
